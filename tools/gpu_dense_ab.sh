#!/bin/bash
# tools/gpu_dense_ab.sh TAG [VAR=VAL ...] -- GPU tests, the dense-event modes (pipelined),
# the same under each VAR=VAL, and a serialized kernel + copy trace of them
set -u
TAG=${1:-dab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
TBF_DEBUG_HOST_PHASES=1 timeout -k 10 300 python3 -u tools/dense_events.py --out "$OUT/dense.json" > "$OUT/phases.log" 2>&1 || { tail -5 "$OUT/phases.log"; exit 1; }
grep '^{' "$OUT/phases.log" | cut -c1-200
for kv in "$@"; do
	echo "== $kv"
	env "$kv" TBF_DEBUG_HOST_PHASES=1 timeout -k 10 300 python3 -u tools/dense_events.py --modes every8,params,dense --steps 4 > "$OUT/phases_$kv.log" 2>&1 || { tail -5 "$OUT/phases_$kv.log"; exit 1; }
	grep '^{' "$OUT/phases_$kv.log" | cut -c1-200
done
TBF_PIPELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/ser" -o run -- \
	python3 -u tools/dense_events.py --modes every8,params,dense --steps 3 > "$OUT/ser.log" 2>&1 || { tail -5 "$OUT/ser.log"; exit 1; }
echo done
