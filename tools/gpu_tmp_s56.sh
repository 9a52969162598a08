#!/bin/bash
# one-off: k_tgctl phase timing with the bus-level traffic ablated (CTL_ABL 1: messages, 2: ctl_block; wrong output)
set -u
O=gpurun_out/r05s56; mkdir -p $O
for v in ctlprof ctlabl1 ctlabl2; do
  TBF_LIB=tunebfree_amd/_variants/libtbf_$v.so timeout -k 10 120 python3 -u tools/dense_events.py --modes dense --steps 2 --warmup 1 > $O/$v.log 2>&1 || { echo $v failed $?; exit 1; }
  echo $v; grep ctlprof $O/$v.log | sort -t" " -k3 -n | head -3 | cut -c1-160; grep mode $O/$v.log | cut -c1-120
done
