#!/bin/bash
# tools/gpu_tgctl_ab.sh TAG -- k_tgctl / k_tonegen durations under dense events (stages
# serialized) for the in-tree library and every variant in tunebfree_amd/_variants
set -u
TAG=${1:-tab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "" tunebfree_amd/_variants/libtbf_*.so; do
	n=$( [ -z "$v" ] && echo base || basename "$v" .so )
	TBF_LIB=${v:-tunebfree_amd/libtbf.so} TBF_PIPELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$n" -o run -- \
		python3 -u tools/dense_events.py --modes dense,every8 --steps 3 > "$OUT/$n.log" 2>&1 || { tail -5 "$OUT/$n.log"; exit 1; }
	python3 - "$OUT/$n" "$n" <<'PY'
import sqlite3, sys, glob, collections
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
d = collections.defaultdict(list)
for nm, s, e in c.execute("select s.kernel_name, k.start, k.end from rocpd_kernel_dispatch k join rocpd_info_kernel_symbol s on k.kernel_id = s.id"):
    d[nm.split("(")[0][:24]].append((e - s) / 1e6)
print(sys.argv[2], {k: (len(v), round(sorted(v)[len(v) // 2], 3)) for k, v in d.items() if "tgctl" in k or "tonegen" in k})
PY
done
