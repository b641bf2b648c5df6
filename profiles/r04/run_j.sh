#!/bin/bash
# round 4, run J: PMC HBM traffic of cfg 4's dominant section (the layer-0 minibatch forward GEMM), merged
# into the committed pmc_traffic.json beside cfg 2's entry; then the cfg-4 line reading it.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j
mkdir -p $O
cd $R
cp profiles/pmc_traffic.json $O/pmc_traffic.json
K="gemm_glds_kernel<1, 4, 1, 1, true, false, 2, false, 4, 2, false>"
cd /tmp && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc4_fetch -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc4_fetch.json 2> $O/pmc4_fetch.err && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc4_write -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc4_write.json 2> $O/pmc4_write.err && \
cd $R && python3 profiles/collect_pmc.py $O/pmc4_fetch $O/pmc4_write --section "gemm_fwd[0]" --kernel "$K" --config 784,512,256,10:60000:1 --out $O/pmc_traffic.json || { echo "pmc failed"; exit 1; }
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --no-cpu-baseline --pmc-json $O/pmc_traffic.json > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo "bench failed"; exit 1; }
tail -1 $O/bench_cfg4.json
echo "run j ok"
