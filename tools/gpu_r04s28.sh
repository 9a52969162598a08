#!/bin/bash
# round 4 session 28: k_whirl serial passes, both products of a step in one packed multiply
# (WH_SERIAL_PK=1 variant, against WH_SERIAL_PIPE=1) -- whirl / chain tests on the variant, then the bench with
# each kernel alone, base and variant alternating, twice
set -u
OUT=gpurun_out/r04s28; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
V=tunebfree_amd/_variants/libtbf_wpk.so
A=tunebfree_amd/_variants/libtbf_wpipe.so
timeout -k 10 400 env TBF_LIB=$V python3 -u -m pytest tests -x -v -s -m gpu -k "whirl or full_chain or steady or bitexact" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 env TBF_LIB=$A python3 bench.py --cpu-baseline 0 --steps 10 --warmup 3 --isolated 1 > $OUT/wpipe_$i.json 2> $OUT/wpipe_$i.err; st wpipe_$i $?; summ $OUT/wpipe_$i.json
timeout -k 10 300 env TBF_LIB=$V python3 bench.py --cpu-baseline 0 --steps 10 --warmup 3 --isolated 1 > $OUT/pk_$i.json 2> $OUT/pk_$i.err; st pk_$i $?; summ $OUT/pk_$i.json
done
