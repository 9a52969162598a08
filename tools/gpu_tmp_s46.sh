#!/bin/bash
# one-off: k_tgctl phase timing with wave start/end stamps; dense-mode kernel trace of the build
set -u
O=gpurun_out/r05s46; mkdir -p $O; export TMPDIR=/tmp
TBF_LIB=tunebfree_amd/_variants/libtbf_ctlprof.so timeout -k 10 120 python3 -u tools/dense_events.py --modes dense --steps 2 --warmup 1 > $O/prof.log 2>&1 || { echo prof failed $?; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 -u tools/dense_events.py --modes dense --steps 4 --warmup 1 > $O/tr.log 2>&1 || { echo tr failed $?; exit 1; }
grep -h "k_tgctl\|k_front\|k_tonegen" $O/tr/run_kernel_stats.csv | cut -c1-120
