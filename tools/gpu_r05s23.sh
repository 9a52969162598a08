#!/bin/bash
# clean timeline of the timed steps, and the device front end's event gate on sparse chunks
set -u
OUT=gpurun_out/r05s23; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --cpu-baseline 0 --check 0 --stage-check 0 --steps 12 --warmup 3 --isolated 0 --steady64 0 --kernel-steps 0 > $OUT/tr.log 2>&1 || exit $?
python3 tools/timeline.py $(find $OUT/tr -name 'run_kernel_trace.csv' | head -1) --out $OUT/timeline.json
for fm in 1024 64; do
	timeout -k 10 400 env TBF_FRONT_MIN=$fm python3 -u tools/dense_events.py --modes sparse256,sparse64,every8,dense --out $OUT/dense_fm$fm.json > $OUT/dense_fm$fm.log 2>&1 || exit $?
	echo "front min $fm"; python3 -c "
import json
for r in json.load(open('$OUT/dense_fm$fm.json'))['rows']: print('  %-10s ev %7d  %.3f ms  host %.3f ms  call %.3f ms' % (r['mode'], r['events_per_step'], r['ms_per_step'], r['host_control_ms_per_step'], r['call_ms_per_step']))"
done
