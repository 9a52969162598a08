#!/bin/bash
# one-off: counting sort by instance in scanChunk: GPU suite, dense host phases, A/B host ms against the previous build
set -u
O=gpurun_out/r05s58; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed $?; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TBF_DEBUG_HOST_PHASES=1 timeout -k 10 120 python3 -u tools/dense_events.py --modes dense --steps 6 --warmup 2 > $O/hp.log 2>&1 || { echo hp failed $?; exit 1; }
grep -E "scan|instances|threads" $O/hp.log | tail -6
for r in 1 2; do
  for v in prev new; do
    L=tunebfree_amd/libtbf.so; [ $v = prev ] && L=tunebfree_amd/_variants/libtbf_prev.so
    TBF_LIB=$L timeout -k 10 200 python3 -u tools/dense_events.py --modes every8,dense --steps 8 --warmup 3 > $O/${v}_$r.log 2>&1 || { echo $v failed $?; exit 1; }
    echo $v $r $(grep mode $O/${v}_$r.log | python3 -c "import sys,json; print(' '.join(r['mode']+' '+str(round(r['ms_per_step'],3))+' host '+str(round(r['host_control_ms_per_step'],3)) for r in map(json.loads, sys.stdin)))")
  done
done
