#!/bin/bash
# Build the committed tree's library into lbfgs-ffnn_amd/build/ab (A/B baseline for run_ab.sh).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive HEAD lbfgs-ffnn_amd include | tar -x -C "$T"
make -C "$T/lbfgs-ffnn_amd" -j8 BUILD="$R/lbfgs-ffnn_amd/build/ab" > /dev/null
rm -rf "$T"
