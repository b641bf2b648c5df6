# Block-level phase stamps of the fused forward GEMM (debug build) + the cfg-2 split plan.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
NS=60000,7500 timeout -k 10 120 python3 -u profiles/ktrace_gemm.py > $O/ktg.txt 2>&1 && \
LBF_SHOW_PLAN=1 timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 20 > $O/plan.json 2> $O/plan.err
echo "rc=$?"
