#!/bin/bash
# tools/iso_cmp.sh TAG [libs...] -- whole-step rate plus each kernel alone (--isolated 1)
# for the in-tree library and the given variant libraries (A/B of kernel changes)
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
run() { # name lib
	local name=$1 lib=$2
	timeout -k 10 300 env TBF_LIB="$lib" python3 bench.py --cpu-baseline 0 --check 2 --steps 5 --warmup 2 --isolated 1 > "$OUT/$name.log" 2>&1
	local rc=$?
	grep '^{' "$OUT/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', round(d['value']/1e9,3), 'err', d['max_err'], 'iso', {k: round(v,3) for k,v in r['kernels_ms_isolated'].items()})"
	return $rc
}
run base tunebfree_amd/libtbf.so || exit $?
for v in "$@"; do run "$(basename $v .so)" "$v" || exit $?; done
exit 0
