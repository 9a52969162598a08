#!/bin/bash
# one-off: k_tgctl rewrite -- GPU suite, phase timing, dense-events step times
set -u
O=gpurun_out/r05s51; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed $?; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TBF_LIB=tunebfree_amd/_variants/libtbf_ctlprof.so timeout -k 10 120 python3 -u tools/dense_events.py --modes dense,every8 --steps 2 --warmup 1 > $O/prof.log 2>&1 || { echo prof failed $?; exit 1; }
grep ctlprof $O/prof.log | sort -t" " -k3 -n | head -20
timeout -k 10 300 python3 -u tools/dense_events.py --modes steady,every8,dense --steps 8 --warmup 3 > $O/de.log 2>&1 || { echo de failed $?; exit 1; }
grep mode $O/de.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 -u tools/dense_events.py --modes dense --steps 10 --warmup 2 > $O/tr.log 2>&1 || { echo tr failed $?; exit 1; }
python3 tools/timeline.py $O/tr/run_kernel_trace.csv > $O/tline.txt 2>&1; tail -10 $O/tline.txt
