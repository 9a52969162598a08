#!/bin/bash
# one-off: dense-mode kernel trace + concurrency timeline of the k_tgctl build
set -u
O=gpurun_out/r05s49; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 -u tools/dense_events.py --modes dense --steps 10 --warmup 2 > $O/tr.log 2>&1 || { echo tr failed $?; exit 1; }
grep mode $O/tr.log | cut -c1-200
python3 tools/timeline.py $O/tr/run_kernel_trace.csv > $O/tline.txt 2>&1; head -40 $O/tline.txt
