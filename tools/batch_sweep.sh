#!/bin/bash
# tools/batch_sweep.sh TAG B1 B2 ... -- per-kernel ms at several batch sizes (tail effects)
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for b in "$@"; do
	timeout -k 10 300 python3 bench.py --batch "$b" --cpu-baseline 0 --check 0 --steps 3 --warmup 1 > "$OUT/b$b.log" 2>&1
	rc=$?
	grep '^{' "$OUT/b$b.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$b', round(d['value']/1e9,3), {k: round(v,3) for k,v in d['roofline']['kernels_ms_per_launch'].items()})"
	[ $rc -ne 0 ] && exit $rc
done
exit 0
