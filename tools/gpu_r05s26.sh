#!/bin/bash
# is k_whirl VALU-bound or latency-bound?  its unloaded time at 4096 / 2048 / 1024 instances
# (4 / 2 / 1 waves per SIMD), and its SQ counters on the current build
set -u
OUT=gpurun_out/r05s26; mkdir -p $OUT; export TMPDIR=/tmp
for b in 4096 2048 1024; do
	timeout -k 10 300 python3 bench.py --batch $b --cpu-baseline 0 --check 0 --stage-check 0 --steps 3 --warmup 1 --isolated 2 --steady64 0 > $OUT/b$b.json 2> $OUT/b$b.err || exit $?
	python3 -c "
import json
d=json.loads([l for l in open('$OUT/b$b.json') if l.startswith('{')][-1])
print('batch $b', '%.4g'%d['value'], '%.2f ms'%d['ms_per_step'], {k:round(v['ms_isolated'],2) for k,v in d['roofline']['kernels'].items()})"
done
PB="--cpu-baseline 0 --check 0 --stage-check 0 --steps 1 --warmup 1 --isolated 0 --steady64 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/psqa -o run --output-format csv -- python3 bench.py $PB > $OUT/psqa.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM -d $OUT/psqb -o run --output-format csv -- python3 bench.py $PB > $OUT/psqb.log 2>&1 || exit $?
echo done
