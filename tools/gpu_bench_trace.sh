# kernel trace of the bench's timed region (no check, no CPU leg)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-benchtrace}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --check 0 --steps 10 --warmup 2 --kernel-steps 1 > $GRAFT_REPO_ROOT/$O/bench.json 2> $GRAFT_REPO_ROOT/$O/bench.err; rc=$?
cd $GRAFT_REPO_ROOT; cut -c1-200 $O/bench.json; exit $rc
