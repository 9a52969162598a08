#!/bin/bash
# configs[3]-style rehearsal on one GPU: two bench ranks (gloo barrier / max-over-ranks), both on device 0
set -u
O=gpurun_out/r05s67; mkdir -p $O
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=2 LOCAL_RANK=0
RANK=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --batch 1024 --steps 5 --warmup 2 --cpu-baseline 0 > $O/r0.log 2>&1 &
p0=$!
RANK=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --batch 1024 --steps 5 --warmup 2 --cpu-baseline 0 > $O/r1.log 2>&1 &
p1=$!
wait $p0; r0=$?; wait $p1; r1=$?
echo rc $r0 $r1
grep '^{' $O/r0.log | tail -1 | cut -c1-400
tail -3 $O/r1.log
