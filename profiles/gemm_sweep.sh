#!/bin/bash
# Sweep the GEMM prefetch depth / k-group variants with the probe (GPU box).
R=${GRAFT_REPO_ROOT:-/root/repo}
for cfg in "LBF_GEMM_PF=1" "LBF_GEMM_PF=2" "LBF_GEMM_PF=3"; do
  env $cfg NS=60000 timeout -k 10 120 python3 $R/profiles/gemm_probe.py 2>&1 | grep "gemm_" | sed "s/^/[$cfg] /"
done
for kw in 1 2; do for pf in 1 2 4; do
  env LBF_GEMM_KW_SMALL=$kw LBF_GEMM_PF_SMALL=$pf NS=7500 timeout -k 10 120 python3 $R/profiles/gemm_probe.py 2>&1 | grep "gemm_" | sed "s/^/[kw=$kw pf=$pf] /"
done; done
