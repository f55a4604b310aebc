#!/bin/bash
# A/B support: build the WORKING TREE with extra compiler flags (a compile-time variant, e.g.
# EXTRA_HIPFLAGS=-DDCT3D_EG_WIN_LINEAR) into ab/<NAME> (git-ignored, travels with the gpurun snapshot):
#   bash tools/ab_variant.sh lin -DDCT3D_EG_WIN_LINEAR
set -e
NAME=$1; shift
cd "$(dirname "$0")/.."
WT=/tmp/ab_var_$NAME
rm -rf $WT && mkdir -p $WT
cp -r Makefile include 3ddctvideoencoding_amd bench.py oracle $WT/
rm -rf $WT/3ddctvideoencoding_amd/lib $WT/build
make -C $WT -j8 all EXTRA_HIPFLAGS="$*" >/dev/null
rm -rf ab/$NAME && mkdir -p ab/$NAME
cp -r $WT/3ddctvideoencoding_amd $WT/bench.py $WT/include $WT/oracle ab/$NAME/
rm -rf $WT
echo "ab/$NAME <- working tree with: $*"
