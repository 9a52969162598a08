set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pipemode}
mkdir -p $O
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], 'value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']), {k: round(v, 2) for k, v in r['kernels_ms_per_launch'].items()})" "$1" "$2"; }
TBF_PIPE_MODE=1 timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "pipelined or full_chain or events or retune_mid" > $O/tests_m1.log 2>&1; rc=$?; tail -2 $O/tests_m1.log; [ $rc -ne 0 ] && exit $rc
for cfg in "0 -" "1 0,0,1,2,2" "1 0,1,1,2,2" "1 0,0,1,1,2" "1 0,1,2,2,2" "0 -" "1 0,0,1,2,2"; do
  set -- $cfg; m=$1; g=$2
  if [ "$g" = "-" ]; then unset TBF_PIPE_GROUPS; else export TBF_PIPE_GROUPS=$g; fi
  TBF_PIPE_MODE=$m timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 1 --stage-check 0 > $O/b_$m_$g.json 2> $O/b.err; rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b.err; exit $rc; }
  summ $O/b_$m_$g.json "mode$m groups$g"
done
