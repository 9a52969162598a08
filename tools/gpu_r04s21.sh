#!/bin/bash
# round 4 session 21: k_whirl constants re-read per sub-block (no SGPR spills, no VGPR spills in the sub-block loop)
# -- whirl tests, A/B against HEAD (twice), whirl phase clocks, SQ counters
set -u
OUT=gpurun_out/r04s21; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu -k "whirl or full_chain or steady or full_size" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --isolated 1 --steps 20 --warmup 5 > $OUT/bench$i.json 2> $OUT/bench$i.err; st bench$i $?
summ $OUT/bench$i.json
timeout -k 10 300 env TBF_LIB=tunebfree_amd/_prof/libtbf_head.so python3 bench.py --cpu-baseline 0 --isolated 1 --steps 20 --warmup 5 > $OUT/bench_head$i.json 2> $OUT/bench_head$i.err; st head$i $?
summ $OUT/bench_head$i.json
done
timeout -k 10 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_whprof.so python3 tools/whirl_prof.py > $OUT/whirl_prof.log 2>&1; st whprof $?
tail -11 $OUT/whirl_prof.log
bash tools/gpu_pmc_probe.sh r04s21/pmc "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" > $OUT/pmc.log 2>&1; st pmc $?
grep -A9 "k_whirl" $OUT/pmc/summary.txt
