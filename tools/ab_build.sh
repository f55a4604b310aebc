#!/bin/bash
# A/B support: build revision REV (default HEAD) in a git worktree and copy the runnable tree to
# ab/<NAME> (git-ignored, travels with the gpurun snapshot), so one GPU call can bench two builds:
#   bash tools/ab_build.sh HEAD~1 base && gpurun -- 'cd ab/base && python bench.py ...; cd ../.. && python bench.py ...'
set -e
REV=${1:-HEAD}; NAME=${2:-base}
cd "$(dirname "$0")/.."
WT=/tmp/ab_wt_$NAME
git worktree remove --force $WT 2>/dev/null || true
git worktree add --detach $WT $REV >/dev/null
make -C $WT -j8 all >/dev/null
rm -rf ab/$NAME && mkdir -p ab/$NAME
cp -r $WT/3ddctvideoencoding_amd $WT/bench.py $WT/include ab/$NAME/
[ -d $WT/oracle ] && cp -r $WT/oracle ab/$NAME/
git worktree remove --force $WT
echo "ab/$NAME <- $(git rev-parse --short $REV)"
