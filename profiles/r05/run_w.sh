#!/bin/bash
# round 5, run W: the vendor fp32 GEMM (torch.matmul, TF32 off) on the headline's GEMM shapes, for scale.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w
mkdir -p $O
cd $R
timeout -k 10 300 python -u profiles/r05/vendor_gemm.py > $O/vendor_gemm.jsonl 2> $O/vendor_gemm.err; echo "rc $?"; cat $O/vendor_gemm.jsonl
