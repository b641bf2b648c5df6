#!/bin/bash
# round 5, run O: phase stamps of the fused forward GEMM + head (debug build, build/ktrace) on the new head,
# with each block's placement (XCC id, CU): main loop and end by XCD and by blocks sharing the CU.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05o
mkdir -p $O
cd $R
NS=7500,60000 timeout -k 10 200 python -u profiles/ktrace_gemm.py > $O/ktrace_gemm.txt 2>&1; echo "ktrace rc $?"; grep -v amdgpu.ids $O/ktrace_gemm.txt
