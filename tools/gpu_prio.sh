# A/B: wave priority of k_rv_core (variants) and stream priority per stage group (env)
set -u
OUT=gpurun_out/${1:-prio}; mkdir -p "$OUT"
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], 'value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), 'kern', {k: round(v, 3) for k, v in r['kernels_ms_per_launch'].items()})" "$1" "$2"; }
run () { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -5 "$OUT/$n.err"; exit 1; }; summ "$OUT/$n.json" "$n"; }
run base X=0
for v in tunebfree_amd/_variants/libtbf_*.so; do run "$(basename $v .so)" TBF_LIB=$v; done
for g in 0 1 2; do run sprio$g TBF_STREAM_PRIO=$g; done
run base2 X=0
