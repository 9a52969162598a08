set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-dense}
mkdir -p $O
timeout -k 10 500 python3 -u tools/dense_events.py --out $O/dense_events.json > $O/dense.log 2>&1; rc=$?; tail -6 $O/dense.log; exit $rc
