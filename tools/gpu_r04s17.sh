#!/bin/bash
# round 4 session 17: k_whirl at 4 waves per SIMD as the default -- every GPU test, the bench
set -u
OUT=gpurun_out/r04s17; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --isolated 1 > $OUT/bench.json 2> $OUT/bench.err; st bench $?
summ $OUT/bench.json
timeout -k 10 300 env TBF_LIB=tunebfree_amd/_prof/libtbf_rg4w3.so python3 bench.py --cpu-baseline 0 --isolated 1 > $OUT/bench_rg4w3.json 2> $OUT/bench_rg4w3.err; st rg4w3 $?
summ $OUT/bench_rg4w3.json
timeout -k 10 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_whprof.so python3 tools/whirl_prof.py > $OUT/whirl_prof.log 2>&1; st whprof $?
tail -12 $OUT/whirl_prof.log
