#!/bin/bash
# one-off: reserve whole CUs for the reverb stream's chain blocks by unused dynamic LDS (TBF_LDS_PAD), with 2 / 3 mid1 sets; same-box A/B
set -u
O=gpurun_out/r05s61; mkdir -p $O
run() { # name env...
  local nm=$1; shift
  env "$@" timeout -k 10 400 python3 -u bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $O/$nm.json 2> $O/$nm.err || { echo $nm failed $?; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$nm.json') if l.startswith('{')][-1]); print('$nm', round(d['value']/1e9,3), round(d['ms_per_step'],2), round(d['steady64']['ms_per_64_blocks'],3), d['max_err'])"
}
run A TBF_MID1_SETS=2
run B TBF_MID1_SETS=2 TBF_LDS_PAD=0,0,106000,0,0,0
run C TBF_MID1_SETS=2 TBF_LDS_PAD=0,0,106000,0,112000,0
run D TBF_MID1_SETS=3 TBF_LDS_PAD=0,0,106000,0,112000,0
run E TBF_MID1_SETS=2 TBF_LDS_PAD=0,0,0,0,112000,0
run A2 TBF_MID1_SETS=2
