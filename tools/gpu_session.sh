#!/bin/bash
# tools/gpu_session.sh -- one gpurun session: parity tests, bench, rocprof stats and PMC
# passes.  Every GPU step has its own time limit; the session stops at the first step
# that faults, aborts, segfaults or times out (exit codes >= 124), and continues past
# ordinary failures (exit 1, e.g. an unknown counter name) so the log shows them.
# usage: tools/gpu_session.sh TAG [steps...]   steps: tests bench ablate stats pmc list
set -u
TAG=${1:-dev}; shift || true
STEPS=${*:-"tests bench stats pmc"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
REPO=$(pwd)
run() { # name timeout cmd...
	local name=$1 to=$2; shift 2
	echo "== $name: $*" | tee -a "$OUT/session.log"
	timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc" | tee -a "$OUT/session.log"
	tail -5 "$OUT/$name.log"
	if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
	return 0
}
BENCHP="--steps 3 --warmup 1 --cpu-baseline 0 --check 0 --blocks 16"
for s in $STEPS; do
	case $s in
	list) run counters 120 rocprofv3 -L ;;
	tests) run tests 900 python3 -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread ;;
	bench) run bench 900 python3 bench.py ;;
	prof) run prof 300 env TBF_LIB=tunebfree_amd/_variants/libtbf_prof.so python3 tools/prof_stages.py ;;
	ablate) for c in 1 2 3 0; do run ablate$c 300 python3 bench.py --chain $c --steps 3 --warmup 1 --cpu-baseline 0 --check 0; done ;;
	stats) run stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 bench.py $BENCHP ;;
	pmc)
		run pmc_a 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/pmc_a" -o run --output-format csv -- python3 bench.py $BENCHP
		run pmc_b 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_FLAT -d "$OUT/pmc_b" -o run --output-format csv -- python3 bench.py $BENCHP
		run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $BENCHP
		run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $BENCHP
		;;
	pmcchain)
		for c in 1 2 3 0; do
			run pmcc$c 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d "$OUT/pmcc$c" -o run --output-format csv -- python3 bench.py $BENCHP --chain $c
		done ;;
	quick) run quick 600 python3 bench.py --cpu-baseline 0 --check 2 --steps 3 --warmup 1 ;;
	variants)
		for v in tunebfree_amd/_variants/libtbf_*.so; do
			run "var_$(basename $v .so)" 300 env TBF_LIB=$v python3 bench.py --cpu-baseline 0 --check 2 --steps 3 --warmup 1
		done ;;
	full)
		BC="--cpu-baseline 0"
		run fstats 600 rocprofv3 --kernel-trace --stats -d "$OUT/fstats" -o run --output-format csv -- python3 bench.py $BC
		run ffetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/ffetch" -o run --output-format csv -- python3 bench.py $BC
		run fwrite 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/fwrite" -o run --output-format csv -- python3 bench.py $BC
		run ftraffic 60 python3 tools/traffic_from_pmc.py "$OUT/ffetch" "$OUT/fwrite" --out "$OUT/traffic.json"
		run fbench 900 python3 bench.py --traffic "$OUT/traffic.json"
		;;
	kpmc)
		BP="--steps 2 --warmup 1 --cpu-baseline 0 --check 0 --blocks 16"
		run kp_a 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/kp_a" -o run --output-format csv -- python3 bench.py $BP
		run kp_b 300 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_LEVEL_VMEM -d "$OUT/kp_b" -o run --output-format csv -- python3 bench.py $BP
		run kp_c 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD -d "$OUT/kp_c" -o run --output-format csv -- python3 bench.py $BP
		run kp_sum 60 python3 tools/pmc_kernels.py 16 "$OUT/kp_a" "$OUT/kp_b" "$OUT/kp_c"
		;;
	calib)
		run calib_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calib_fetch" -o run --output-format csv -- python3 tools/calib_pmc.py
		run calib_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/calib_write" -o run --output-format csv -- python3 tools/calib_pmc.py
		;;
	*) echo "unknown step $s" ;;
	esac
done
echo "session done"
