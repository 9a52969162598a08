# host-control threading experiment: dense events at 4096 instances, serial loop vs
# threaded stepping at T workers (T=1: the threaded code inline on the calling thread)
set -o pipefail
O=gpurun_out/${1:-hostpar}
mkdir -p $O
echo "== serial" >> $O/log
TBF_HOST_SERIAL=1 timeout -k 10 120 python3 -u tools/dense_events.py --modes dense --steps 4 >> $O/log 2>&1 || exit $?
for T in ${THREADS:-1 2 16}; do
  echo "== T=$T" >> $O/log
  TBF_HOST_THREADS=$T TBF_DEBUG_HOST_PHASES=1 timeout -k 10 120 python3 -u tools/dense_events.py --modes dense --steps 4 >> $O/log 2>&1 || exit $?
done
