#!/bin/bash
# tools/gpu_rvc.sh TAG [pytest -k expr | none] -- GPU parity tests, then the default bench
# twice (kernels alone and pipelined) and every build variant in tunebfree_amd/_variants.
set -u
TAG=${1:-rvc}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
KARG=(); [ -n "$K" ] && KARG=(-k "$K")
if [ "$K" != "none" ]; then
	timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread "${KARG[@]}" > "$OUT/tests.log" 2>&1
	rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
fi
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], 'value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'kern', {k: round(v, 3) for k, v in r['kernels_ms_per_launch'].items()}, 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" "$1" "$2"; }
run() { # name [env...]
	local n=$1; shift
	env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 --isolated 1 > "$OUT/$n.json" 2> "$OUT/$n.err"
	local rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/$n.err"; exit $rc; }
	summ "$OUT/$n.json" "$n"
}
run base
for v in tunebfree_amd/_variants/libtbf_*.so; do
	[ -e "$v" ] || continue
	run "$(basename "$v" .so)" TBF_LIB=$v
done
run base2
