#!/bin/bash
# round 4, run T: evidence (traces, PMC, two-loop, every bench line) on the final tree of round 4 (suite, smoke, driver-shape and
# 400-iteration cfg 2, the 7500-row shard, cfg 4, deep and cfg-3 lines, kernel traces, PMC, two-loop).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04t
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; }
B bench_driver --steps 20 --warmup 5
B bench_400 --steps 400 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
B bench_cfg4 --solver slbfgs --steps 6
B bench_cfg4_b --solver slbfgs --steps 6 --no-cpu-baseline
B bench_deep_m10 --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 10 --line-search armijo --init cuda --steps 200 --no-cpu-baseline
B bench_cfg3 --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline
timeout -k 10 300 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop.jsonl 2> $O/two_loop.err || { echo "two-loop failed"; exit 1; }
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv && \
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv || { echo "kstats failed"; exit 1; }
cp profiles/pmc_traffic.json $O/pmc_traffic.json
K="gemm_glds_kernel<2, 2, 2, 2, true, false, 3, false, 2"
cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc_write.json 2> $O/pmc_write.err && \
cd $R && python3 profiles/collect_pmc.py $O/pmc_fetch $O/pmc_write --section "gemm_fwd[0]" --kernel "$K" --config 784,128,10:60000:1 --out $O/pmc_traffic.json || { echo "pmc failed"; exit 1; }
K4="gemm_glds_kernel<1, 4, 1, 1, true, false, 2, false, 4, 2, false>"
cd /tmp && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc4_fetch -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc4_fetch.json 2> $O/pmc4_fetch.err && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc4_write -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc4_write.json 2> $O/pmc4_write.err && \
cd $R && python3 profiles/collect_pmc.py $O/pmc4_fetch $O/pmc4_write --section "gemm_fwd[0]" --kernel "$K4" --config 784,512,256,10:60000:1 --out $O/pmc_traffic.json || { echo "pmc4 failed"; exit 1; }
echo "run t ok"
