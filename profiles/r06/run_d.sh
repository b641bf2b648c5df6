#!/bin/bash
# Run D (round 6): where the two-loop's sweeps lose their last ~10 % — the ring-stride
# micro-benchmark (profiles/micro/ring_ld.hip), the two-loop bench, and PMC FETCH / WRITE of the Gram and combine
# sweeps at m = 50 (n = 10.49M); then PMC FETCH / WRITE of the cfg-3 and cfg-5 dominant dW GEMMs (item 7).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 profiles/micro/ring_ld.hip -o $O/ring_ld > $O/ring_ld_build.txt 2>&1 || { echo "build failed"; cat $O/ring_ld_build.txt; exit 1; }
timeout -k 10 180 $O/ring_ld > $O/ring_ld.txt 2>&1 || { echo "ring_ld failed"; tail $O/ring_ld.txt; exit 1; }
cat $O/ring_ld.txt
timeout -k 10 240 python -u bench_two_loop.py --m 10,50 > $O/two_loop.jsonl 2> $O/two_loop.err || { echo "two-loop failed"; tail -5 $O/two_loop.err; exit 1; }
cat $O/two_loop.jsonl | python3 -c "import json,sys; [print('two_loop m', d['m'], d['roofline']['frac'], d['gram_us'], d['hist_coef_us'], d['combine_us'], d['gram_GBs'], d['combine_GBs']) for d in map(json.loads, sys.stdin)]"
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/pmc2l_$c -o run -- python3 $R/bench_two_loop.py --m 50 --iters 4 > $O/pmc2l_$c.json 2> $O/pmc2l_$c.err || { echo "pmc two-loop failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/pmc3_$c -o run -- python3 $R/bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 10 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc3_$c.json 2> $O/pmc3_$c.err || { echo "pmc cfg3 failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc5_$c -o run -- python3 $R/bench.py --data regression --samples 1000000 --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --steps 2 --warmup 1 --no-cpu-baseline --device-warmup 0 > $O/pmc5_$c.json 2> $O/pmc5_$c.err || { echo "pmc cfg5 failed"; exit 1; }
done
cd $R
P=profiles/collect_pmc.py
python3 $P $O/pmc2l_FETCH_SIZE $O/pmc2l_WRITE_SIZE --section gram_sweep --kernel "gram_kernel<4, true>" --config "two_loop:10489857:m50" --out $O/pmc_two_loop.json --largest-grid && \
python3 $P $O/pmc2l_FETCH_SIZE $O/pmc2l_WRITE_SIZE --section combine_sweep --kernel "combine_kernel<8, true>" --config "two_loop:10489857:m50" --out $O/pmc_two_loop.json && \
python3 $P $O/pmc3_FETCH_SIZE $O/pmc3_WRITE_SIZE --section "gemm_dw[0]" --kernel "gemm_glds_kernel<2, 2, 2, 2, false, false, 2," --config "784,128,64,10:60000:1" --out $O/pmc_dw.json --largest-grid && \
python3 $P $O/pmc5_FETCH_SIZE $O/pmc5_WRITE_SIZE --section "gemm_dw[0]" --kernel "gemm_glds_kernel<2, 2, 2, 2, false, false, 2," --config "4096,2048,1024,1:1000000:1" --out $O/pmc_dw.json --largest-grid || echo "collect failed"
cat $O/pmc_two_loop.json $O/pmc_dw.json
echo "run d ok"
