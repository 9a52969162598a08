#!/bin/bash
# round 4 session 18: network tap addresses formed in the previous write phase -- reverb
# tests, A/B against HEAD (twice), network phase clocks
set -u
OUT=gpurun_out/r04s18; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
timeout -k 10 600 python3 -u -m pytest tests -x -v -s -m gpu -k "reverb or full_chain or stage_taps or steady or full_size" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --isolated 1 > $OUT/bench$i.json 2> $OUT/bench$i.err; st bench$i $?
summ $OUT/bench$i.json
timeout -k 10 300 env TBF_LIB=tunebfree_amd/_prof/libtbf_head.so python3 bench.py --cpu-baseline 0 --isolated 1 > $OUT/bench_head$i.json 2> $OUT/bench_head$i.err; st head$i $?
summ $OUT/bench_head$i.json
done
timeout -k 10 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_rvlprof.so python3 tools/rvl_prof.py > $OUT/rvl_prof.log 2>&1; st rvl $?
tail -16 $OUT/rvl_prof.log
