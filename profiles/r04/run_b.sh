#!/bin/bash
# round 4, run B: suite after the tail revert / K2 removal; A/B of the deferred S-LBFGS gradient reduction;
# rocprofv3 kernel traces of cfg 2, the 7500-row shard and cfg 4; PMC traffic of the cfg-2 forward GEMM.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04b
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; }
B bench_driver --steps 20 --warmup 5
B bench_400 --steps 400 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
B bench_cfg4 --solver slbfgs --steps 6 --no-cpu-baseline
LBF_SLBFGS_DEFER=0 B bench_cfg4_nodefer --solver slbfgs --steps 6 --no-cpu-baseline
B bench_cfg4_b --solver slbfgs --steps 6 --no-cpu-baseline
LBF_SLBFGS_DEFER=0 B bench_cfg4_nodefer_b --solver slbfgs --steps 6 --no-cpu-baseline
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv && \
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv || { echo "kstats failed"; exit 1; }
K="gemm_glds_kernel<2, 2, 2, 2, true, false, 3, false, 2"
cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_write.json 2> $O/pmc_write.err && \
cd $R && python3 profiles/collect_pmc.py $O/pmc_fetch $O/pmc_write --section "gemm_fwd[0]" --kernel "$K" --config 784,128,10:60000:1 --out $O/pmc_traffic.json || { echo "pmc failed"; exit 1; }
echo "main steps ok"
KT_N=7500 timeout -k 10 120 python3 profiles/ktrace.py > $O/ktrace_7500.txt 2>&1 && \
KT_N=60000 timeout -k 10 120 python3 profiles/ktrace.py > $O/ktrace_60000.txt 2>&1 || { echo "ktrace failed"; exit 1; }
echo "ktrace ok"
