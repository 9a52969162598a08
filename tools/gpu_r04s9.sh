#!/bin/bash
# round 4 session 9: full GPU suite; host phase timings of the dense-event modes
set -u
OUT=gpurun_out/r04s9; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
timeout -k 10 900 python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; st tests $?
tail -3 $OUT/tests.log
TBF_DEBUG_HOST_PHASES=1 timeout -k 10 300 python3 -u tools/dense_events.py --modes params,dense --steps 3 --warmup 1 --instances 4096 > $OUT/phases.log 2>&1; st phases $?
grep -E "stepChunkFront|mode" $OUT/phases.log | tail -12
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --isolated 1 > $OUT/bench.json 2> $OUT/bench.err; st bench $?
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $OUT/bench.json
timeout -k 10 200 env TBF_LIB=tunebfree_amd/_prof/libtbf_whprof.so python3 tools/whirl_prof.py > $OUT/whirl_prof.log 2>&1; st whprof $?
tail -11 $OUT/whirl_prof.log
