#!/bin/bash
# one-off: padded bus-level rows with 16-B sc1 row loads in ctl_block: GPU suite, same-box A/B against HEAD's k_tgctl
set -u
O=gpurun_out/${TAG}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed $?; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base new; do
    L=tunebfree_amd/libtbf.so; [ $v = base ] && L=tunebfree_amd/_variants/libtbf_base.so
    TBF_LIB=$L timeout -k 10 200 python3 -u tools/dense_events.py --modes every8,dense --steps 8 --warmup 3 > $O/${v}_$r.log 2>&1 || { echo $v failed $?; exit 1; }
    echo $v $r $(grep mode $O/${v}_$r.log | python3 -c "import sys,json; print(' '.join(r['mode']+' '+str(round(r['ms_per_step'],3))+' host '+str(round(r['host_control_ms_per_step'],3)) for r in map(json.loads, sys.stdin)))")
  done
done
