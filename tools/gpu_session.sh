#!/bin/bash
# tools/gpu_session.sh TAG [steps...] -- one gpurun session of measurements for profiles/.
# Every GPU step has its own time limit; the session stops at the first step that faults,
# aborts or times out (exit codes >= 124) and goes on past ordinary failures.
#   tests   the GPU parity suite
#   full    rocprofv3 --kernel-trace --stats of the default bench without its parity-check
#           engines (so every dispatch is full size) and the full-size kernel summary
#   pmc     per-kernel PMC profile (FETCH_SIZE, WRITE_SIZE, two SQ passes: separate runs) ->
#           kernel_pmc.json, which bench.py's roofline reads
#   fbench  the driver's bench (20 steps, 5 warmup) with that profile
#   cfg     secondary lines: configs[1] at 256 instances, configs[4] shape, dense events, RT latency
#   steady  the bench with the steady chunk capped at 256 .. 2048 blocks (footprint vs speed)
#   front   the device front end's event gate (sparse / dense modes) and its host phases
#   split   k_whirl vs k_whirl_split (96 kHz, 2048 instances, RT periods)
#   wscale  unloaded kernel times at 4096 / 2048 / 1024 instances
#   bench   the default bench without the CPU leg
#   ab:V=X  the default bench with environment switch V=X
#   prof    k_rv_core_lds / k_whirl / k_tonegen phase clocks (tools/build_prof.sh variants)
#   ctlprof k_tgctl phase clocks under dense / every-8 events, with the bus-level traffic
#           ablated (tools/build_prof.sh variants; the ablations' output is wrong)
#   ctlab:LIB  same-box A/B of dense / every-8 events: the in-tree library against LIB,
#           alternating, two runs each (LIB: a build of the round's start, for example)
#   calib   PMC byte counters on known aligned / misaligned streams
#   smoke   __graft_entry__.smoke() (the driver's round-end check)
#   world2  two bench ranks through bench.py's own launcher, both on device 0 (rehearsal)
set -u
TAG=${1:-dev}; shift || true
STEPS=${*:-"tests pmc fbench full"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name timeout cmd...
	local name=$1 to=$2; shift 2
	echo "== $name: $*" | tee -a "$OUT/session.log"
	timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc" | tee -a "$OUT/session.log"
	tail -3 "$OUT/$name.log"
	if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
	return 0
}
NC="--cpu-baseline 0 --check 0 --stage-check 0"
for s in $STEPS; do
	case $s in
	tests) run tests 900 python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread ;;
	full)
		run fstats 300 rocprofv3 --kernel-trace --stats -d "$OUT/fstats" -o run --output-format csv -- python3 bench.py $NC
		run fsum 60 python3 tools/kernel_stats.py "$(find "$OUT/fstats" -name 'run_kernel_trace.csv' | head -1)" --out "$OUT/kernel_stats_full.json"
		# the concurrency profile of the timed steps alone (no kernel-time, isolated or steady64 passes)
		run tstats 300 rocprofv3 --kernel-trace -d "$OUT/tstats" -o run --output-format csv -- python3 bench.py $NC --steps 12 --warmup 3 --isolated 0 --steady64 0 --kernel-steps 0
		run tline 60 python3 tools/timeline.py "$(find "$OUT/tstats" -name 'run_kernel_trace.csv' | head -1)" --out "$OUT/timeline.json"
		;;
	pmc) # the per-kernel PMC profile bench.py's roofline reads: FETCH_SIZE, WRITE_SIZE and two
		# SQ passes (each its own run), full-size launches, then tools/kernel_pmc.py
		PB="$NC --steps 1 --warmup 1 --isolated 0 --steady64 0"
		run plist 60 rocprofv3 -L
		T32=""; grep -q "SQ_INSTS_VALU_TRANS_F32" "$OUT/plist.log" && T32=SQ_INSTS_VALU_TRANS_F32
		run pfetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pfetch" -o run --output-format csv -- python3 bench.py $PB
		run pwrite 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pwrite" -o run --output-format csv -- python3 bench.py $PB
		run psqa 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/psqa" -o run --output-format csv -- python3 bench.py $PB
		run psqb 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 $T32 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d "$OUT/psqb" -o run --output-format csv -- python3 bench.py $PB
		run psum 60 python3 tools/kernel_pmc.py "$OUT/pfetch" "$OUT/pwrite" "$OUT/psqa" "$OUT/psqb" --blocks ${BLOCKS:-2048} --launch-blocks ${LAUNCH_BLOCKS:-512} --out "$OUT/kernel_pmc.json"
		;;
	fbench) # the driver's bench (20 steps, 5 warmup) with this session's PMC profile
		run fbench 900 python3 bench.py --steps 20 --warmup 5 --pmc "$OUT/kernel_pmc.json"
		cp "$OUT/fbench.log" "$OUT/bench.json" ;;
	cfg)
		run cfg2 300 python3 bench.py --workload cfg2 --batch 256 --cpu-baseline 0 --check 8
		run cfg5 300 python3 bench.py --workload cfg5 --cpu-baseline 0 --check 8
		run dense 500 python3 -u tools/dense_events.py --out "$OUT/dense_events.json"
		run rt 300 python3 -u tools/rt_latency.py --out "$OUT/rt_latency.json"
		run rt_nospin 300 python3 -u tools/rt_latency.py --spin-ms 0 --warmup 200 --out "$OUT/rt_latency_nospin.json"
		;;
	steady) # the bench at 2048-block steps with the steady chunk capped (stage-buffer footprint vs speed)
		for c in 256 512 1024 2048; do
			run "steady$c" 400 env TBF_STEADY_CHUNK=$c python3 bench.py --cpu-baseline 0 --check 0 --stage-check 0 --steps 10 --warmup 3 --isolated 0 --steady64 0
		done ;;
	front) # the device front end: sparse and dense modes at two event gates, then its host phases
		for fm in 1024 64; do
			run "front_fm$fm" 400 env TBF_FRONT_MIN=$fm python3 -u tools/dense_events.py --modes sparse256,sparse64,every8,dense --out "$OUT/dense_fm$fm.json"
		done
		run front_phases 300 env TBF_DEBUG_HOST_PHASES=1 python3 -u tools/dense_events.py --modes dense --steps 4 --warmup 2 ;;
	split) # k_whirl against k_whirl_split: 96 kHz, 2048 instances, real-time periods
		for sp in 0 1; do
			run "split${sp}_cfg5" 300 env TBF_WHIRL_SPLIT=$sp python3 bench.py --workload cfg5 --cpu-baseline 0 --check 4 --steps 3 --warmup 1 --steady64 0 --isolated 2
			run "split${sp}_b2048" 300 env TBF_WHIRL_SPLIT=$sp python3 bench.py --batch 2048 --cpu-baseline 0 --check 4 --steps 5 --warmup 2 --steady64 0 --isolated 2
			run "split${sp}_rt" 300 env TBF_WHIRL_SPLIT=$sp python3 -u tools/rt_latency.py --out "$OUT/rt_split$sp.json"
		done ;;
	wscale) # unloaded kernel times at 4096 / 2048 / 1024 instances (waves per SIMD vs latency)
		for b in 4096 2048 1024; do
			run "wscale$b" 300 python3 bench.py --batch $b --cpu-baseline 0 --check 0 --stage-check 0 --steps 3 --warmup 1 --isolated 2 --steady64 0
		done ;;
	bench) run bench 300 python3 bench.py --cpu-baseline 0 ;;
	bench2048x2) # two driver-length benches (A/B baseline on one box)
		run bench_a 400 python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5
		run bench_b 400 python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 ;;
	prof) # phase clocks of k_rv_core_lds and k_whirl (build variants from tools/*_prof_patch.py)
		run rvl_prof 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_rvlprof.so python3 tools/rvl_prof.py
		run whirl_prof 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_whprof.so python3 tools/whirl_prof.py
		run tg_prof 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_tgprof.so python3 tools/phase_prof.py --chain 1 ;;
	ctlprof) # printed by a few workgroups per launch: cycles of the stage, message, active-list and removal phases
		for v in ctlprof ctlabl1 ctlabl2; do
			run "$v" 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_$v.so python3 -u tools/dense_events.py --modes dense,every8 --steps 2 --warmup 1
		done ;;
	ctlab:*)
		lib=${s#ctlab:}
		for r in 1 2; do
			run "ctlab_base_$r" 200 env TBF_LIB=$lib python3 -u tools/dense_events.py --modes every8,dense --steps 8 --warmup 3
			run "ctlab_new_$r" 200 python3 -u tools/dense_events.py --modes every8,dense --steps 8 --warmup 3
		done ;;
	calib) # FETCH_SIZE / WRITE_SIZE of known streams: aligned and 64 B misaligned 8-B/lane reads and writes
		run calib_f 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calib_f" -o run --output-format csv -- python3 tools/calib_pmc.py 2 0,2,1,3
		run calib_w 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/calib_w" -o run --output-format csv -- python3 tools/calib_pmc.py 2 0,2,1,3 ;;
	smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
	world2) run world2 400 env TBF_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 2 --batch 1024 --cpu-baseline 0 --steps 3 --warmup 1 ;;
	ab:*) # ab:VAR=VALUE -- the default bench with one environment switch (A/B)
		kv=${s#ab:}
		run "ab_${kv//[^A-Za-z0-9_]/_}" 300 env "$kv" python3 bench.py --cpu-baseline 0 ;;
	*) echo "unknown step $s" ;;
	esac
done
echo "session done"
