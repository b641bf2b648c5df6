# Shader clock over the fused forward GEMM's main loop (debug build) and one PMC pass of MFMA busy
# cycles over the cfg-2 bench (counters alone, no trace domains).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
NS=60000 timeout -k 10 120 python3 -u profiles/ktrace_gemm.py > $O/ktg.txt 2>&1 && \
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $O/pmc_mfma.json 2> $O/pmc_mfma.err
echo "rc=$?"
