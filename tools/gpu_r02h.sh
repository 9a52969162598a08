set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02h
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r02h/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02h/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/rt_latency.py --periods 3000 --out gpurun_out/r02h/rt_latency.json > gpurun_out/r02h/rt.log 2>&1; rc=$?; tail -5 gpurun_out/r02h/rt.log; exit $rc
