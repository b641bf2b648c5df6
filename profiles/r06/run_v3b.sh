#!/bin/bash
# Run V3-2 (round 6): evidence on the round's final tree, part 2 — the two-loop bench (m = 10 / 20 / 50), kernel traces
# (cfg 2 driver shape, the 7500-row shard, cfg 4) with live statistics, PMC FETCH / WRITE of the cfg-2 and cfg-4
# dominant forwards.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06v3
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop.jsonl 2> $O/two_loop.err || { echo "two-loop failed"; exit 1; }
cat $O/two_loop.jsonl | python3 -c "import json,sys; [print('two_loop m', d['m'], d['roofline']['frac'], d['gram_us'], d['hist_coef_us'], d['combine_us'], d['gram_GBs'], d['combine_GBs']) for d in map(json.loads, sys.stdin)]"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2l -o run -- python3 $R/bench_two_loop.py --m 50 --iters 4 > $O/kt2l.json 2> $O/kt2l.err || { echo "prof failed"; exit 1; }
for m in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc60_$m -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc60_$m.json 2> $O/pmc60_$m.err || { echo "pmc failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc4_$m -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc4_$m.json 2> $O/pmc4_$m.err || { echo "pmc failed"; exit 1; }
done
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv && \
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv && \
python3 profiles/kstats_live.py $O/kt2l/run_kernel_trace.csv --out $O/kt2l_live.csv || echo "kstats failed"
P=profiles/collect_pmc.py
python3 $P $O/pmc60_FETCH_SIZE $O/pmc60_WRITE_SIZE --section "gemm_fwd[0]" --kernel "gemm_glds_kernel<2, 2, 2, 2, true, false, 3, false, 2" --config "784,128,10:60000:1" --out $O/pmc_traffic.json && \
python3 $P $O/pmc4_FETCH_SIZE $O/pmc4_WRITE_SIZE --section "gemm_fwd[0]" --kernel "gemm_glds_kernel<1, 4, 1, 1, true, false, 2, false, 4, 2, false>" --config "784,512,256,10:60000:1" --out $O/pmc_traffic.json || echo "collect failed"
head -4 $O/kt60000_live.csv
echo "run v3-2 ok"
