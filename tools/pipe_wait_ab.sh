#!/bin/bash
# tools/pipe_wait_ab.sh TAG "w0,w1,w2,w3,w4" ... -- whole-step rate per TBF_PIPE_WAIT table
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for w in "$@"; do
	f="$OUT/w_${w//,/_}.log"
	timeout -k 10 300 env TBF_PIPE_WAIT="$w" python3 bench.py --cpu-baseline 0 --check 2 --steps 10 --warmup 2 > "$f" 2>&1 || exit $?
	grep '^{' "$f" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('wait=$w', round(d['value']/1e9,3), round(d['ms_per_step'],3), 'err', d['max_err'], {k: round(v,3) for k,v in r['kernels_ms_per_launch'].items()})"
done
