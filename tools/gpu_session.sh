#!/bin/bash
# tools/gpu_session.sh TAG [steps...] -- one gpurun session of measurements for profiles/.
# Every GPU step has its own time limit; the session stops at the first step that faults,
# aborts or times out (exit codes >= 124) and goes on past ordinary failures.
#   tests   the GPU parity suite
#   full    rocprofv3 --kernel-trace --stats of the default bench without its parity-check
#           engines (so every dispatch is full size), FETCH_SIZE / WRITE_SIZE passes ->
#           traffic.json, the full-size kernel summary, then the default bench with traffic
#   kpmc    per-kernel SQ counters (occupancy, waits, LDS activity and bank conflicts)
#   cfg     secondary lines: configs[1] at 256 instances, configs[4] shape, dense events
#   iso     the default bench with each kernel also timed alone (--isolated 1)
#   bench   the default bench without the CPU leg
#   ab:V=X  the default bench with environment switch V=X
#   prof    k_rv_core_lds / k_whirl / k_tonegen phase clocks (tools/build_prof.sh variants)
#   calib   PMC byte counters on known aligned / misaligned streams
set -u
TAG=${1:-dev}; shift || true
STEPS=${*:-"tests full kpmc"}
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
		run ffetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/ffetch" -o run --output-format csv -- python3 bench.py $NC
		run fwrite 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/fwrite" -o run --output-format csv -- python3 bench.py $NC
		run ftraffic 60 python3 tools/traffic_from_pmc.py "$OUT/ffetch" "$OUT/fwrite" --blocks ${BLOCKS:-2048} --out "$OUT/traffic.json"
		run fbench 900 python3 bench.py --steps 20 --warmup 5 --traffic "$OUT/traffic.json"
		cp "$OUT/fbench.log" "$OUT/bench.json"
		;;
	kpmc)
		BP="--steps 2 --warmup 1 $NC --blocks 16"
		run kp_a 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/kp_a" -o run --output-format csv -- python3 bench.py $BP
		run kp_b 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/kp_b" -o run --output-format csv -- python3 bench.py $BP
		run kp_c 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD -d "$OUT/kp_c" -o run --output-format csv -- python3 bench.py $BP
		run kp_sum 60 python3 tools/pmc_kernels.py 16 "$OUT/kp_a" "$OUT/kp_b" "$OUT/kp_c"
		cp "$OUT/kp_sum.log" "$OUT/pmc_kernels.txt"
		;;
	cfg)
		run cfg2 300 python3 bench.py --workload cfg2 --batch 256 --cpu-baseline 0 --check 8
		run cfg5 300 python3 bench.py --workload cfg5 --cpu-baseline 0 --check 8
		run dense 500 python3 -u tools/dense_events.py --out "$OUT/dense_events.json"
		run rt 300 python3 -u tools/rt_latency.py --out "$OUT/rt_latency.json"
		;;
	iso) run iso 300 python3 bench.py --steps 20 --warmup 5 --isolated 1 --cpu-baseline 0 ;;
	prof) # phase clocks of k_rv_core_lds and k_whirl (build variants from tools/*_prof_patch.py)
		run rvl_prof 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_rvlprof.so python3 tools/rvl_prof.py
		run whirl_prof 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_whprof.so python3 tools/whirl_prof.py
		run tg_prof 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_tgprof.so python3 tools/phase_prof.py --chain 1 ;;
	calib) # FETCH_SIZE / WRITE_SIZE of known streams: aligned and 64 B misaligned 8-B/lane reads and writes
		run calib_f 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calib_f" -o run --output-format csv -- python3 tools/calib_pmc.py 2 0,2,1,3
		run calib_w 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/calib_w" -o run --output-format csv -- python3 tools/calib_pmc.py 2 0,2,1,3 ;;
	bench) run bench 300 python3 bench.py --cpu-baseline 0 ;;
	fbench:*) # fbench:DIR -- the driver's bench (20 steps, 5 warmup) with DIR/traffic.json
		d=${s#fbench:}
		run fbench 900 python3 bench.py --steps 20 --warmup 5 --traffic "$d/traffic.json"
		cp "$OUT/fbench.log" "$OUT/bench.json" ;;
	ab:*) # ab:VAR=VALUE -- the default bench with one environment switch (A/B)
		kv=${s#ab:}
		run "ab_${kv//[^A-Za-z0-9_]/_}" 300 env "$kv" python3 bench.py --cpu-baseline 0 ;;
	*) echo "unknown step $s" ;;
	esac
done
echo "session done"
