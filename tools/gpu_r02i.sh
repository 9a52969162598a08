set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02i}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "device_control_programs" > $O/ctl.log 2>&1; rc=$?; tail -15 $O/ctl.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
TBF_HOST_CONTROL=1 timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread -k "not device_control" > $O/tests_hostctl.log 2>&1; rc=$?; tail -3 $O/tests_hostctl.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 -u tools/dense_events.py --out $O/dense_events.json > $O/dense.log 2>&1; rc=$?; tail -6 $O/dense.log; exit $rc
