#!/bin/bash
# tools/gpu_test_ab.sh TAG "NAME:VAR=V ..." ... -- GPU parity tests, then tools/gpu_envab.sh with the given env variants
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -15 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_envab.sh "$TAG" "$@"
