#!/bin/bash
# round 5, run AE: evidence on the final tree of the round (run Y + the tail kernels' abort-flag change, run AC). Whole
# suite, smoke; bench lines (driver shape with the CPU baseline, 400 iterations, the 7500-row shard single and
# through a 1-rank communicator, cfg 3, deep Armijo m = 10, cfg 4 with its CPU baseline, cfg 5); the two-loop
# microbenchmark; kernel traces (cfg 2 driver shape, 7500 rows, cfg 4) and PMC FETCH/WRITE (cfg 2, cfg 4);
# the forward GEMM's per-block stamps with placement (debug build, raw per-block CSV).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ae
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
B() { n=$1; shift; timeout -k 10 240 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('cpu_baseline',{}).get('value'))"; }
B bench_driver --steps 20 --warmup 5
B bench_400 --steps 400 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
B bench_7500_comm1 --steps 400 --samples 7500 --no-cpu-baseline --comm1
B bench_cfg3 --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline
B bench_deep_m10 --dims 784,256,128,64,10 --acts relu,relu,relu,linear --line-search armijo --init cuda --steps 200 --no-cpu-baseline
B bench_cfg4 --solver slbfgs --steps 6
B bench_cfg5 --data regression --samples 1000000 --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --steps 3 --warmup 1 --no-cpu-baseline --device-warmup 0
timeout -k 10 240 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop.jsonl 2> $O/two_loop.err || { echo "two-loop failed"; exit 1; }
cat $O/two_loop.jsonl | python3 -c "import json,sys; [print('two_loop m', d['m'], d['roofline']['frac'], d['gram_us'], d['hist_coef_us'], d['combine_us']) for d in map(json.loads, sys.stdin)]"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err || { echo "prof failed"; exit 1; }
for m in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc60_$m -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc60_$m.json 2> $O/pmc60_$m.err || { echo "pmc failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc4_$m -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc4_$m.json 2> $O/pmc4_$m.err || { echo "pmc failed"; exit 1; }
done
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv && \
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv || echo "kstats failed"
head -4 $O/kt60000_live.csv
if [ -f lbfgs-ffnn_amd/build/ktrace/liblbfgs_amd_abi3.so ]; then
KT_RAW=$O/ktrace_blocks NS=7500,60000 timeout -k 10 200 python -u profiles/ktrace_gemm.py > $O/ktrace_gemm.txt 2>&1; echo "ktrace rc $?"
fi
echo "run ae ok"
