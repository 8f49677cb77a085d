#!/bin/bash
# Build the library of a commit (default HEAD) into vision_transformer_detector_amd/libvtd_prev.so,
# the "prev" side of tools/experiments/r5_ab.sh (a git worktree under /tmp; no repo files touched).
set -e
REV=${1:-HEAD}
ROOT=$(git -C "$(dirname "$0")/.." rev-parse --show-toplevel)
WT=/tmp/vtd_prev_wt
rm -rf $WT; git -C $ROOT worktree prune
git -C $ROOT worktree add -q --detach $WT $REV
make -C $WT/vision_transformer_detector_amd/csrc -j8 BUILD=$WT/build/csrc > /tmp/vtd_prev_build.log 2>&1
cp $WT/vision_transformer_detector_amd/libvtd.so $ROOT/vision_transformer_detector_amd/libvtd_prev.so
git -C $ROOT worktree remove --force $WT
echo "libvtd_prev.so <- $(git -C $ROOT rev-parse --short $REV)"
