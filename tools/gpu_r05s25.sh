#!/bin/bash
set -u
OUT=gpurun_out/r05s25; mkdir -p $OUT; export TMPDIR=/tmp
python3 -c "
import ctypes
h=ctypes.CDLL('/opt/rocm/lib/libamdhip64.so')
lo,hi=ctypes.c_int(),ctypes.c_int()
print('stream priority range', h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo),ctypes.byref(hi)), lo.value, hi.value)"
TAG=r05s25 bash tools/gpu_abl.sh rvc16 mp16 both16 || exit $?
B="--cpu-baseline 0 --check 0 --stage-check 0 --steps 5 --warmup 2 --steady64 0"
timeout -k 10 300 env TBF_GROUP_PRIO=0,0,0 python3 bench.py $B > $OUT/prio0.json 2> $OUT/prio0.err || exit $?
python3 -c "
import json
d=json.loads([l for l in open('$OUT/prio0.json') if l.startswith('{')][-1])
print('prio0', '%.4g'%d['value'], '%.2f ms'%d['ms_per_step'])"
