#!/bin/bash
# host front-end time under dense events by host worker count
set -u
OUT=gpurun_out/r05s34; mkdir -p $OUT; export TMPDIR=/tmp
nproc; python3 -c "import os; print('sched cpus', len(os.sched_getaffinity(0)))"
for th in 16 8 4; do
	timeout -k 10 300 env TBF_HOST_THREADS=$th python3 -u tools/dense_events.py --modes every8,dense --out $OUT/dense_t$th.json > /dev/null 2>&1 || exit $?
	python3 -c "
import json
for r in json.load(open('$OUT/dense_t$th.json'))['rows']: print('threads $th  %-8s %.3f ms  host %.3f ms' % (r['mode'], r['ms_per_step'], r['host_control_ms_per_step']))"
done
