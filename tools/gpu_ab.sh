#!/bin/bash
# tools/gpu_ab.sh TAG [pytest -k expr] -- GPU parity tests, then the in-tree library's bench
# (kernels alone and pipelined) and every build variant in tunebfree_amd/_variants (A/B).
set -u
TAG=${1:-ab}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
KARG=(); [ -n "$K" ] && KARG=(-k "$K")
if [ "$K" != "none" ]; then
	timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread "${KARG[@]}" > "$OUT/tests.log" 2>&1
	rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
fi
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], 'value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'kern', {k: round(v, 3) for k, v in r['kernels_ms_per_launch'].items()}, 'iso', {k: round(v, 3) for k, v in (r['kernels_ms_isolated'] or {}).items()})" "$1" "$2"; }
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 --isolated 1 ${BENCH_ARGS:-} > "$OUT/base.json" 2> "$OUT/base.err"
rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/base.err"; exit $rc; }
summ "$OUT/base.json" base
for v in tunebfree_amd/_variants/libtbf_*.so; do
	[ -e "$v" ] || continue
	n=$(basename "$v" .so)
	TBF_LIB=$v timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 --isolated 1 ${BENCH_ARGS:-} > "$OUT/$n.json" 2> "$OUT/$n.err"
	rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/$n.err"; exit $rc; }
	summ "$OUT/$n.json" "$n"
done
# the in-tree library once more (run-to-run spread)
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 --isolated 1 ${BENCH_ARGS:-} > "$OUT/base2.json" 2> "$OUT/base2.err" && summ "$OUT/base2.json" base2
