set -u
OUT=gpurun_out/pipe; mkdir -p $OUT
[ "${SKIP_TESTS:-0}" = 1 ] || { timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }; }
tail -2 $OUT/tests.log
for i in 1 2; do
for pm in 1 0; do
timeout -k 10 300 env TBF_PIPELINE=$pm python3 bench.py --cpu-baseline 0 --check 2 --steps 10 --warmup 2 > $OUT/b_${pm}_${i}.log 2>&1 || exit 1
grep '^{' $OUT/b_${pm}_${i}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('pipe=$pm', round(d['value']/1e9,3), d['ms_per_step'], 'err', d['max_err'], {k: round(v,3) for k,v in r['kernels_ms_per_launch'].items()})"
done; done
