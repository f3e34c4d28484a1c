#!/bin/bash
# Build libsfmfeat.so of a git revision into ab_head/<rev>/ (git-ignored; it travels to the GPU
# box with the tree) for same-box A/B runs: SFMFEAT_LIB=ab_head/<rev>/libsfmfeat.so.
set -eu
cd "$(dirname "$0")/.."
rev=$(git rev-parse --short "${1:-HEAD}")
wt=/tmp/sfm_wt_$rev
[ -d "$wt" ] || git worktree add -f "$wt" "$rev" > /dev/null
make -C "$wt/sfmfromscratch_amd/csrc" -j8 OUTDIR="$PWD/ab_head/$rev" > /dev/null
echo "ab_head/$rev/libsfmfeat.so"
