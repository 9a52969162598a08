# GPU parity tests, stage profile, bench with kernels alone, and the streaming reverb core for A/B
set -u
mkdir -p gpurun_out/lds && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/lds/tests.log 2>&1
rc=$?; tail -3 gpurun_out/lds/tests.log; [ $rc -ne 0 ] && exit $rc
TBF_LIB=tunebfree_amd/_prof/libtbf_prof.so timeout -k 10 200 python3 tools/prof_stages.py --batch 4096 --blocks 64 > gpurun_out/lds/prof.txt 2>&1 || exit 1
grep -E "total|rv_lds|rv_core" gpurun_out/lds/prof.txt
for v in 1 0; do
TBF_RV_LDS=$v timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 --isolated 1 > gpurun_out/lds/iso$v.json 2> gpurun_out/lds/iso$v.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lds/iso$v.json') if l.startswith('{')][-1]); r=d['roofline']; print('RV_LDS=$v', d['ms_per_step'], d['max_err'], {k: round(x,3) for k,x in r['kernels_ms_per_launch'].items()}, {k: round(x,3) for k,x in r['kernels_ms_isolated'].items()})"
done
