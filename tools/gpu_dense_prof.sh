set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-denseprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o dense -- python3 $GRAFT_REPO_ROOT/tools/dense_events.py --modes ${MODES:-dense,every8} --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; tail -3 $O/prof.log; find $O/prof -name "*stats*" | head; exit $rc
