# Round 2, run C: bench lines for cfg 3 / cfg 5 / m = 100 / cfg 4 (S-LBFGS), kernel traces of m = 100 and
# cfg 4, and the PMC passes north_star names (MFMA busy for the GEMMs at cfg 2 and cfg 5; HBM FETCH /
# WRITE for the two-loop kernels at n = 10.49 M and the cfg-2 forward GEMM). One counter group per pass.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02c
mkdir -p $O
cd $R
B="python3 $R/bench.py --no-cpu-baseline"
timeout -k 10 120 python -u bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err && \
timeout -k 10 120 python -u bench.py --m 100 --no-cpu-baseline > $O/bench_cfg2_m100.json 2> $O/bench_cfg2_m100.err && \
timeout -k 10 300 python -u bench.py --solver slbfgs --steps 2 --warmup 1 > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --cpu-iters 2 --cpu-samples 400 > $O/bench_cfg5.json 2> $O/bench_cfg5.err && \
cd /tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_m100 -o run -- $B --m 100 --steps 50 > $O/kt_m100.json 2> $O/kt_m100.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg4 -o run -- $B --solver slbfgs --steps 1 --warmup 1 > $O/kt_cfg4.json 2> $O/kt_cfg4.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma_cfg2 -o run -- $B --steps 20 > $O/pmc_mfma_cfg2.json 2> $O/pmc_mfma_cfg2.err && \
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma_cfg5 -o run -- $B --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 2 --warmup 1 > $O/pmc_mfma_cfg5.json 2> $O/pmc_mfma_cfg5.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_cfg2 -o run -- $B --steps 5 --warmup 2 > $O/pmc_fetch_cfg2.json 2> $O/pmc_fetch_cfg2.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_cfg2 -o run -- $B --steps 5 --warmup 2 > $O/pmc_write_cfg2.json 2> $O/pmc_write_cfg2.err && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_2loop -o run -- python3 $R/bench_two_loop.py --m 10,50 > $O/pmc_fetch_2loop.jsonl 2> $O/pmc_fetch_2loop.err && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_2loop -o run -- python3 $R/bench_two_loop.py --m 10,50 > $O/pmc_write_2loop.jsonl 2> $O/pmc_write_2loop.err && \
cd $R && \
python3 profiles/kstats_live.py $O/kt_m100/run_kernel_trace.csv --out $O/kt_m100_live.csv > /dev/null && \
python3 profiles/r02/pmc_summary.py $O/pmc_mfma_cfg2 --match gemm_glds > $O/pmc_mfma_cfg2.txt && \
python3 profiles/r02/pmc_summary.py $O/pmc_mfma_cfg5 --match gemm_glds > $O/pmc_mfma_cfg5.txt && \
python3 profiles/r02/pmc_summary.py $O/pmc_fetch_cfg2 $O/pmc_write_cfg2 --match gemm_glds tail_ combine > $O/pmc_traffic_cfg2.txt && \
python3 profiles/r02/pmc_summary.py $O/pmc_fetch_2loop $O/pmc_write_2loop --match gram_kernel combine_kernel hist_step fold_rows > $O/pmc_traffic_2loop.txt
echo "rc=$?"
