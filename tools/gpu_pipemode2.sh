set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pipemode2}
mkdir -p $O
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], 'value %.4g ms/step %.3f err %s' % (d['value'], d['ms_per_step'], d['max_err']))" "$1" "$2"; }
i=0
for cfg in "0 -" "1 0,1,1,2,2" "0 -" "1 0,1,1,2,2" "0 -" "1 0,1,1,2,2" "1 0,1,1,1,2" "1 0,0,0,1,2"; do
  i=$((i+1)); set -- $cfg; m=$1; g=$2
  if [ "$g" = "-" ]; then unset TBF_PIPE_GROUPS; else export TBF_PIPE_GROUPS=$g; fi
  TBF_PIPE_MODE=$m timeout -k 10 300 python3 bench.py --cpu-baseline 0 --check 1 --stage-check 0 --steps 10 > $O/b$i.json 2> $O/b.err; rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b.err; exit $rc; }
  summ $O/b$i.json "mode$m groups$g"
done
