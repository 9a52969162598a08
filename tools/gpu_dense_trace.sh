# kernel trace (no copy/API tracing) of the dense-events workload, for the per-stream timeline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-densetrace}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o dense -- python3 $GRAFT_REPO_ROOT/tools/dense_events.py --modes ${MODES:-dense} --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; grep mode $O/prof.log; exit $rc
