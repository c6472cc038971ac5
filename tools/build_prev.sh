#!/bin/bash
# Build the committed HEAD's library into tools/lib/libprev.so (travels to the GPU box; git-ignored) (A/B baseline).
cd "$(dirname "$0")/.." || exit 2
R=$PWD
rm -rf /tmp/dm_prev_wt /tmp/dm_prev_build && git worktree add -q /tmp/dm_prev_wt HEAD || exit 1
make -s -C /tmp/dm_prev_wt/diffusion-models-pytorch_amd/csrc -j8 OUT=${PREV_OUT:-$R/tools/lib/libprev.so} BUILD=/tmp/dm_prev_build
rc=$?
git worktree remove --force /tmp/dm_prev_wt
exit $rc
