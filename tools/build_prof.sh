#!/bin/bash
# tools/build_prof.sh -- build the profiling variants (never the product) into tunebfree_amd/_prof:
# k_rv_core_lds phase clocks (rvl_prof_patch.py), k_whirl (whirl_prof_patch.py), k_tonegen
# (phase_prof_patch.py tonegen); k_tgctl phase clocks and bus-level ablations (tbf_ctl.hip's
# TBF_CTL_PROF / CTL_ABL switches); each links the in-tree objects of the other sources.
set -e
cd "$(dirname "$0")/../tunebfree_amd"
make -s libtbf.so
mkdir -p _prof
python3 ../tools/rvl_prof_patch.py _prof/rvlprof.hip
python3 ../tools/whirl_prof_patch.py _prof/whprof.hip
python3 ../tools/phase_prof_patch.py tonegen _prof/tgprof.hip
for v in rvlprof whprof tgprof; do
	make -s variant NAME=$v VSRC=_prof/$v.hip
	mv _variants/libtbf_$v.so _prof/
	rm -rf _variants/$v
done
# k_tgctl: phase clocks (ctlprof), and with the messages' / ctl_block's bus-level traffic
# ablated (ctlabl1 / ctlabl2: timing only, wrong output)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-gpu-flush-denormals-to-zero"
OBJ="_build/tbf_render.o _build/tbf_calib.o _build/tbf_tpl.o _build/tbf_engine.o _build/tbf_init.o _build/tbf_control.o _build/tbf_config.o"
for v in "ctlprof:-DTBF_CTL_PROF" "ctlabl1:-DTBF_CTL_PROF -DCTL_ABL=1" "ctlabl2:-DTBF_CTL_PROF -DCTL_ABL=2"; do
	name=${v%%:*}
	/opt/rocm/bin/hipcc $F ${v#*:} -c csrc/tbf_ctl.hip -o _prof/$name.o
	/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o _prof/libtbf_$name.so _prof/$name.o $OBJ
done
ls _prof/*.so
