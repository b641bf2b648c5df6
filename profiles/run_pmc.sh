# PMC HBM-traffic passes for the bench's dominant kernel (separate FETCH_SIZE / WRITE_SIZE runs; no
# trace domains beside --pmc), then the per-launch bytes into profiles/pmc_traffic.json.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
K="gemm_glds_kernel<2, 2, 2, 2, true, false, 3, false, 2"
cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_write.json 2> $O/pmc_write.err && \
python3 $R/profiles/collect_pmc.py $O/pmc_fetch $O/pmc_write --section "gemm_fwd[0]" --kernel "$K" --config 784,128,10:60000:1 --out $O/pmc_traffic.json
echo "rc=$?"
