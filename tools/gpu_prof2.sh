# stage profile (profiling build in tunebfree_amd/_prof) at batch 256 and 4096, then the bench with kernels alone
mkdir -p gpurun_out/prof && export TMPDIR=/tmp
for b in 256 4096; do TBF_LIB=tunebfree_amd/_prof/libtbf_prof.so timeout -k 10 200 python3 tools/prof_stages.py --batch $b --blocks 64 > gpurun_out/prof/b$b.txt 2>&1 || exit 1; done
cat gpurun_out/prof/b256.txt gpurun_out/prof/b4096.txt
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 --isolated 1 > gpurun_out/prof/iso.json 2> gpurun_out/prof/iso.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/prof/iso.json') if l.startswith('{')][-1]); r=d['roofline']; print(d['ms_per_step'], r['kernels_ms_per_launch'], r['kernels_ms_isolated'])"
