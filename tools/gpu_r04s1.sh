#!/bin/bash
# round 4 session 1: network-kernel phase clocks, k_whirl phase clocks, PMC attribution checks
set -u
OUT=gpurun_out/r04s1; mkdir -p $OUT; export TMPDIR=/tmp
st() { echo "== $1 rc=$2"; if [ $2 -ge 124 ]; then exit $2; fi; }
timeout -k 10 400 python3 -u -m pytest tests -x -v -m gpu -k "front_end or whirl_control" --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; st tests $?
TBF_LIB=tunebfree_amd/_variants/libtbf_rvlprof.so timeout -k 10 200 python3 tools/rvl_prof.py > $OUT/rvl_prof.txt 2>&1; st rvl $?
TBF_LIB=tunebfree_amd/_variants/libtbf_whprof.so timeout -k 10 200 python3 tools/whirl_prof.py > $OUT/whirl_prof.txt 2>&1; st wh $?
NC="--cpu-baseline 0 --check 0 --stage-check 0"
TBF_RV_PERSIST=0 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_np -o run --output-format csv -- python3 bench.py $NC > $OUT/f_np.log 2>&1; st f_np $?
TBF_RV_PERSIST=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_np -o run --output-format csv -- python3 bench.py $NC > $OUT/w_np.log 2>&1; st w_np $?
timeout -k 10 60 python3 tools/traffic_from_pmc.py $OUT/f_np $OUT/w_np --out $OUT/traffic_np.json > $OUT/t_np.log 2>&1; st t_np $?
TBF_PIPELINE=0 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_ser -o run --output-format csv -- python3 bench.py $NC > $OUT/f_ser.log 2>&1; st f_ser $?
TBF_PIPELINE=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_ser -o run --output-format csv -- python3 bench.py $NC > $OUT/w_ser.log 2>&1; st w_ser $?
timeout -k 10 60 python3 tools/traffic_from_pmc.py $OUT/f_ser $OUT/w_ser --out $OUT/traffic_ser.json > $OUT/t_ser.log 2>&1; st t_ser $?
echo done
