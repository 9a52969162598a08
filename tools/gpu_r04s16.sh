#!/bin/bash
# round 4 session 14: k_whirl with a 9.8 KB LDS footprint (filter outputs in the serial pass,
# DPP histories, LDS-free angle replay) -- tests, then A/B: default (4 rings per group),
# 2 rings per group, 2 rings at 4 waves per SIMD, HEAD
set -u
OUT=gpurun_out/r04s16; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
for i in 1 2; do
for v in default rg2w4 noang; do
  if [ $v = default ]; then L=""; else L="TBF_LIB=tunebfree_amd/_prof/libtbf_$v.so"; fi
  timeout -k 10 300 env $L python3 bench.py --cpu-baseline 0 --isolated 1 > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err; st ${v}_$i $?
  summ $OUT/bench_${v}_$i.json
done
done
timeout -k 10 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_whprof.so python3 tools/whirl_prof.py > $OUT/whirl_prof.log 2>&1; st whprof $?
tail -12 $OUT/whirl_prof.log
timeout -k 10 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_whprof_w4.so python3 tools/whirl_prof.py > $OUT/whirl_prof_w4.log 2>&1; st whprof_w4 $?
tail -12 $OUT/whirl_prof_w4.log
