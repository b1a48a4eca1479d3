#!/bin/bash
# gpurun with the tree's identity stamped into BUILD_COMMIT first (the GPU box
# gets no .git; tools/pmc_fold.py records it in the evidence files).
# usage: tools/gpurun.sh <timeout s> '<command>'
cd "$(dirname "$0")/.." || exit 1
git describe --always --dirty --abbrev=12 > BUILD_COMMIT
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
