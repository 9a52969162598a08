#!/bin/bash
# tools/build_prof.sh -- build the profiling variants (never the product) into tunebfree_amd/_prof:
# k_rv_core_lds phase clocks (rvl_prof_patch.py), k_whirl (whirl_prof_patch.py), k_tonegen
# (phase_prof_patch.py tonegen); each links the in-tree objects of the other sources.
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
ls _prof/*.so
