#!/bin/bash
# host phases of the device front end under dense events
set -u
OUT=gpurun_out/r05s31; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 env TBF_DEBUG_HOST_PHASES=1 python3 -u tools/dense_events.py --modes every8,dense --steps 4 --warmup 2 > $OUT/dense.log 2> $OUT/dense.err || exit $?
cat $OUT/dense.log
grep -E "clean|stepChunkFront|threads" $OUT/dense.err | tail -24
