#!/bin/bash
# tools/gpu_abx.sh TAG VARIANT... -- same-box A/B with parity on every variant.
# Each library (base = the in-tree tunebfree_amd/libtbf.so, then every named variant
# tunebfree_amd/_variants/libtbf_NAME.so) first runs the parity gate (the full-chain bench
# batch and the odd-batch mixed scenarios, with and without forced serial paths, bit for
# bit against the CPU oracle); a variant that fails it is not timed.  The passing ones are
# then timed alternately, ROUNDS times each (default 2), with the default bench's kernels
# alone and pipelined.  The summary (summary.txt) carries each variant's parity result beside
# its times.  Options by environment: ROUNDS, BENCH_ARGS, PARITY_K (pytest -k expression).
# A variant NAME=VAR=VALUE runs the in-tree library with the environment variable VAR=VALUE
# (e.g. g000112=TBF_PIPE_GROUPS=0,0,0,1,1,2).
set -u
TAG=${1:-abx}; shift || true
VARS=("base" "$@")
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
K=${PARITY_K:-"test_gpu_full_chain_bench or test_gpu_full_chain_odd_batch or test_gpu_forced_serial or test_gpu_vs_committed or test_gpu_whirl_control_functions or test_gpu_parameter_sweep"}
lib() { case "$1" in base|*=*) echo tunebfree_amd/libtbf.so ;; *) echo "tunebfree_amd/_variants/libtbf_$1.so" ;; esac; }
venv() { case "$1" in *=*) echo "${1#*=}" ;; *) echo "TBF_ABX_NONE=1" ;; esac; }
declare -A PAR
for vv in "${VARS[@]}"; do
	v=${vv%%=*}
	L=$(lib "$vv")
	env "$(venv "$vv")" TBF_LIB=$L timeout -k 10 400 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread -k "$K" \
		> "$OUT/parity_$v.log" 2>&1
	rc=$?
	if [ $rc -ge 124 ]; then echo "STOP: parity of $v rc=$rc"; tail -5 "$OUT/parity_$v.log"; exit $rc; fi
	PAR[$v]=$( [ $rc -eq 0 ] && grep -Eo '[0-9]+ passed' "$OUT/parity_$v.log" | tail -1 || echo "FAILED rc=$rc" )
	echo "parity $v: ${PAR[$v]}" | tee -a "$OUT/summary.txt"
done
B="--cpu-baseline 0 --check 2 --stage-check 0 --steps ${STEPS:-10} --warmup 3 --isolated 2 --steady64 0 ${BENCH_ARGS:-}"
for r in $(seq 1 "${ROUNDS:-2}"); do
	for vv in "${VARS[@]}"; do
		v=${vv%%=*}
		case "${PAR[$v]}" in FAILED*) continue ;; esac
		env "$(venv "$vv")" TBF_LIB=$(lib "$vv") timeout -k 10 300 python3 bench.py $B > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err"
		rc=$?
		if [ $rc -ne 0 ]; then echo "bench $v rc=$rc"; tail -5 "$OUT/${v}_$r.err"; [ $rc -ge 124 ] && exit $rc; continue; fi
		python3 - "$OUT/${v}_$r.json" "$v" "$r" "${PAR[$v]}" <<'EOF' | tee -a "$OUT/summary.txt"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = d["roofline"]["kernels"]
print(f"{sys.argv[2]} r{sys.argv[3]}: {d['ms_per_step']:.2f} ms/step ({d['value']:.4g}) max_err {d['max_err']} "
      f"exact {d['bit_exact_frac']} parity [{sys.argv[4]}] alone",
      {k: round(v["ms_isolated"], 3) for k, v in ks.items()},
      "rendered", {k: round(v["ms_as_rendered"], 2) for k, v in ks.items()})
EOF
	done
done
echo "abx done"
