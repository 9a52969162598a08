#!/bin/bash
# round 4 session 39: steady chunks of up to 2048 blocks (TBF_STEADY_MAX=2048 build) --
# steady / full-chain tests on it, then the bench at 2048-block steps against the default
# 1024, alternating, twice (the driver's step counts)
set -u
OUT=gpurun_out/r04s39; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']))" $1; }
V=tunebfree_amd/_variants/libtbf_s2048.so
timeout -k 10 400 env TBF_LIB=$V python3 -u -m pytest tests -x -v -s -m gpu -k "steady or full_chain or full_size" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -2 $OUT/tests.log; st tests $rc
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 400 env TBF_LIB=$V python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 --blocks 2048 > $OUT/b2048_$i.json 2> $OUT/b2048_$i.err; st b2048_$i $?; summ $OUT/b2048_$i.json
timeout -k 10 400 python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $OUT/b1024_$i.json 2> $OUT/b1024_$i.err; st b1024_$i $?; summ $OUT/b1024_$i.json
done
