set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02j}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 -u tools/dense_events.py --out $O/dense_events.json > $O/dense.log 2>&1; rc=$?; tail -6 $O/dense.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 2 --stage-check 0 > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 600 $O/bench.json; exit $rc
