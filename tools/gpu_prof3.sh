# stage profile of the profiling build (tunebfree_amd/_prof) at 256 and 4096 instances
mkdir -p gpurun_out/prof3 && export TMPDIR=/tmp
for b in 256 4096; do TBF_LIB=tunebfree_amd/_prof/libtbf_prof.so timeout -k 10 200 python3 tools/prof_stages.py --batch $b --blocks 64 > gpurun_out/prof3/b$b.txt 2>&1 || exit 1; done
cat gpurun_out/prof3/b256.txt gpurun_out/prof3/b4096.txt | grep -v amdgpu.ids
