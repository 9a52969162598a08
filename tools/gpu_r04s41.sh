#!/bin/bash
# round 4 session 41: smoke () and the default bench (no flags), with its wall time
set -u
OUT=gpurun_out/r04s41; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; st smoke $?
t0=$(date +%s.%N)
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
t1=$(date +%s.%N)
echo "bench wall $(python3 -c "print(round($t1 - $t0, 1))") s" | tee $OUT/wall.txt; st bench $rc
