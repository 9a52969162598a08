#!/bin/bash
# tools/gpu_pmc_probe.sh TAG "COUNTERS" ["COUNTERS" ...] -- one rocprofv3 --pmc pass per
# counter set over a short bench (16 blocks, no checks), then the per-kernel summary.
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BP="--steps 2 --warmup 1 --cpu-baseline 0 --check 0 --stage-check 0 --blocks 16"
i=0; dirs=()
for set in "$@"; do
	i=$((i+1))
	timeout -k 10 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py $BP > "$OUT/p$i.log" 2>&1
	rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; [ $rc -ge 124 ] && exit $rc; continue; }
	dirs+=("$OUT/p$i")
done
python3 tools/pmc_kernels.py 16 "${dirs[@]}" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
