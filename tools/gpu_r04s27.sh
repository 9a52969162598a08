#!/bin/bash
# round 4 session 27: k_mixpre at 16 instances per workgroup (256 workgroups; MP_CB=16
# variant, with the whirl serial pipelining) -- the GPU suite on the variant, then the
# bench with each kernel alone: wpipe (MP_CB 32) and mp16 alternating, twice
set -u
OUT=gpurun_out/r04s27; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" $1; }
A=tunebfree_amd/_variants/libtbf_wpipe.so
B=tunebfree_amd/_variants/libtbf_mp16.so
timeout -k 10 600 env TBF_LIB=$B python3 -u -m pytest tests -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 env TBF_LIB=$A python3 bench.py --cpu-baseline 0 --steps 10 --warmup 3 --isolated 1 > $OUT/wpipe_$i.json 2> $OUT/wpipe_$i.err; st wpipe_$i $?; summ $OUT/wpipe_$i.json
timeout -k 10 300 env TBF_LIB=$B python3 bench.py --cpu-baseline 0 --steps 10 --warmup 3 --isolated 1 > $OUT/mp16_$i.json 2> $OUT/mp16_$i.err; st mp16_$i $?; summ $OUT/mp16_$i.json
done
