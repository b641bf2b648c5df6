#!/bin/bash
# round 4, run L: tail_reduce loads in flight, bench --device-warmup; split-K forward + row head at the 8-rank shard (7500 rows of cfg 2) against the fused
# 32 x 128 forward (LBF_FWD_SPLIT / LBF_FWD_SPLIT_BM, A/B only), with the row head's one-row-ahead loads.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04l
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('evals_per_iter'), d.get('kernel_ms_per_step'))"; }
B base_a --steps 400 --samples 7500 --no-cpu-baseline
LBF_FWD_SPLIT=4 LBF_FWD_SPLIT_BM=128 B s4_128 --steps 400 --samples 7500 --no-cpu-baseline
LBF_FWD_SPLIT=2 LBF_FWD_SPLIT_BM=64 B s2_64 --steps 400 --samples 7500 --no-cpu-baseline
LBF_FWD_SPLIT=2 LBF_FWD_SPLIT_BM=32 B s2_32 --steps 400 --samples 7500 --no-cpu-baseline
LBF_FWD_SPLIT=3 LBF_FWD_SPLIT_BM=128 B s3_128 --steps 400 --samples 7500 --no-cpu-baseline
LBF_FWD_SPLIT=6 LBF_FWD_SPLIT_BM=128 B s6_128 --steps 400 --samples 7500 --no-cpu-baseline
B base_b --steps 400 --samples 7500 --no-cpu-baseline
# tail_reduce with 24 slab loads per column in flight (one round for cfg 2's 82 dW slabs) against 8
B c2_u24_a --steps 400 --no-cpu-baseline
LBF_TAIL_U=8 B c2_u8_a --steps 400 --no-cpu-baseline
B c2_u24_b --steps 400 --no-cpu-baseline
LBF_TAIL_U=8 B c2_u8_b --steps 400 --no-cpu-baseline
# the driver's shape with and without 300 untimed evaluations at the initial point first
B drv_a --steps 20 --warmup 5 --no-cpu-baseline
B drv_w_a --steps 20 --warmup 5 --no-cpu-baseline --device-warmup 300
B drv_b --steps 20 --warmup 5 --no-cpu-baseline
B drv_w_b --steps 20 --warmup 5 --no-cpu-baseline --device-warmup 300
cd /tmp
export LBF_FWD_SPLIT=4 LBF_FWD_SPLIT_BM=128
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500_s4 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500_s4.json 2> $O/kt7500_s4.err || { echo "prof failed"; exit 1; }
export LBF_FWD_SPLIT=2 LBF_FWD_SPLIT_BM=64
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500_s2 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500_s2.json 2> $O/kt7500_s2.err || { echo "prof failed"; exit 1; }
unset LBF_FWD_SPLIT LBF_FWD_SPLIT_BM
cd $R
python3 profiles/kstats_live.py --spec $O/kt7500_s4/run_kernel_trace.csv --out $O/kt7500_s4_live.csv && \
python3 profiles/kstats_live.py --spec $O/kt7500_s2/run_kernel_trace.csv --out $O/kt7500_s2_live.csv || { echo "kstats failed"; exit 1; }
head -8 $O/kt7500_s4_live.csv $O/kt7500_s2_live.csv
echo "run l ok"
