# dense-events variants: pipelining modes, chunks per call
set -o pipefail
O=gpurun_out/${1:-densevar}
mkdir -p $O
run () { echo "== $1" >> $O/log; shift; env "$@" timeout -k 10 120 python3 -u tools/dense_events.py --modes dense --steps 6 >> $O/log 2>&1; }
run default TBF_X=0 || exit 1
run pipe0 TBF_PIPE_MODE=0 || exit 1
run nopipe TBF_PIPELINE=0 || exit 1
echo "== blocks128" >> $O/log
timeout -k 10 120 python3 -u tools/dense_events.py --modes dense --steps 6 --blocks 128 >> $O/log 2>&1 || exit 1
