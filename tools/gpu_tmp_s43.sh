#!/bin/bash
# one-off: PMC passes over the dense-events mode (k_tgctl / k_front / k_tonegen under control deltas)
set -u
O=gpurun_out/r05s43; mkdir -p $O; export TMPDIR=/tmp
D="python3 -u tools/dense_events.py --modes dense --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY -d $O/pa -o run --output-format csv -- $D > $O/pa.log 2>&1 || { echo pa failed $?; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES -d $O/pb -o run --output-format csv -- $D > $O/pb.log 2>&1 || { echo pb failed $?; exit 1; }
echo done
