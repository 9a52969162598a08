#!/bin/bash
# one-off: same-box A/B of the control-kernel build against HEAD's (dense, every8), alternating
set -u
O=gpurun_out/r05s53; mkdir -p $O
for r in 1 2 3; do
  for v in base new; do
    L=tunebfree_amd/libtbf.so; [ $v = base ] && L=tunebfree_amd/_variants/libtbf_base.so
    TBF_LIB=$L timeout -k 10 200 python3 -u tools/dense_events.py --modes every8,dense --steps 8 --warmup 3 > $O/${v}_$r.log 2>&1 || { echo $v failed $?; exit 1; }
    echo $v $r $(grep mode $O/${v}_$r.log | python3 -c "import sys,json; print(' '.join(r['mode']+' '+str(round(r['ms_per_step'],3)) for r in map(json.loads, sys.stdin)))")
  done
done
