#!/bin/bash
# tools/build_prev.sh [REV] -- build libtbf.so of git revision REV (default HEAD) into
# tunebfree_amd/_variants/libtbf_prev.so, the baseline of the next tools/gpu_ab.sh run.
set -eu
REV=${1:-HEAD}
D=$(mktemp -d /tmp/tbfprev.XXXX)
git archive "$REV" tunebfree_amd include | tar -x -C "$D"
make -C "$D/tunebfree_amd" -j8 libtbf.so > "$D/build.log" 2>&1
mkdir -p tunebfree_amd/_variants
cp "$D/tunebfree_amd/libtbf.so" tunebfree_amd/_variants/libtbf_prev.so
rm -rf "$D"
echo "tunebfree_amd/_variants/libtbf_prev.so <- $REV"
