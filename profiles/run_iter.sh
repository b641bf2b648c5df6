# Iteration loop: GPU tests, fused-GEMM phase stamps, cfg-2 and 7500-row benches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
NS=60000,7500 timeout -k 10 120 python3 -u profiles/ktrace_gemm.py > $O/ktg.txt 2>&1 && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 200 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 200 > $O/bench.json 2> $O/bench.err
echo "rc=$?"
LBF_SHOW_PLAN=1 timeout -k 10 60 python -u bench.py --no-cpu-baseline --steps 5 > /dev/null 2> $O/plan.err
LBF_NO_FOLD=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 200 > $O/bench_nofold.json 2> $O/bench_nofold.err
