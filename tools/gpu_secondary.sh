# secondary measurements of the current build: dense events, config-5 shape, real-time latency
set -u
O=gpurun_out/${1:-secondary}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/dense_events.py --out $O/dense_events.json > $O/dense.log 2>&1; rc=$?; tail -6 $O/dense.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --workload cfg5 --cpu-baseline 0 --check 8 > $O/cfg5.json 2> $O/cfg5.err; rc=$?; [ $rc -ne 0 ] && { tail -5 $O/cfg5.err; exit $rc; }
python3 -c "import json; d=json.loads([l for l in open('$O/cfg5.json') if l.startswith('{')][-1]); print('cfg5', d['value'], d['ms_per_step'], d['max_err'], d['bit_exact_frac'])"
timeout -k 10 300 python3 -u tools/rt_latency.py --out $O/rt_latency.json > $O/rt.log 2>&1; rc=$?; tail -4 $O/rt.log; exit $rc
