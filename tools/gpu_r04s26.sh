#!/bin/bash
# round 4 session 26: k_whirl serial passes with the next group's reads ahead
# (WH_SERIAL_PIPE=1 variant) -- whirl / chain tests on the variant, then the bench with
# each kernel alone, base and variant alternating, twice
set -u
OUT=gpurun_out/r04s26; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
V=tunebfree_amd/_variants/libtbf_wpipe.so
timeout -k 10 400 env TBF_LIB=$V python3 -u -m pytest tests -x -v -s -m gpu -k "whirl or full_chain or steady or bitexact" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --steps 10 --warmup 3 --isolated 1 > $OUT/base_$i.json 2> $OUT/base_$i.err; st base_$i $?; summ $OUT/base_$i.json
timeout -k 10 300 env TBF_LIB=$V python3 bench.py --cpu-baseline 0 --steps 10 --warmup 3 --isolated 1 > $OUT/pipe_$i.json 2> $OUT/pipe_$i.err; st pipe_$i $?; summ $OUT/pipe_$i.json
done
