#!/bin/bash
# stage-group stream priorities under dense / every-8 events: default (reverb group high) against others, alternating
set -u
O=gpurun_out/${1:-prio}; mkdir -p $O
for r in 1 2; do
  for v in default "-1,-1,0" "-1,0,0"; do
    nm=$(echo "p$v" | tr -c 'A-Za-z0-9\n' '_')
    if [ "$v" = default ]; then E=""; else E="TBF_GROUP_PRIO=$v"; fi
    env $E timeout -k 10 200 python3 -u tools/dense_events.py --modes every8,dense --steps 8 --warmup 3 > $O/${nm}_$r.log 2>&1 || { echo $nm failed $?; exit 1; }
    echo $v $r $(grep mode $O/${nm}_$r.log | python3 -c "import sys,json; print(' '.join(r['mode']+' '+str(round(r['ms_per_step'],3)) for r in map(json.loads, sys.stdin)))")
  done
done
