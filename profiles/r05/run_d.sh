#!/bin/bash
# round 5, run D: the wave-split-K direct-load 32 x 128 GEMM (gemm_wsk_kernel): whole GPU suite, then A/B
# against the LDS-DMA loop (LBF_NO_WSK=1) at the 8-rank shard and cfg 4, interleaved
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05d
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit 1; }
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('kernel_ms_per_step'))"; }
for rep in 1 2; do
B s7500_wsk_$rep --steps 400 --samples 7500 --no-cpu-baseline
LBF_NO_WSK=1 B s7500_lds_$rep --steps 400 --samples 7500 --no-cpu-baseline
done
for rep in 1 2; do
B cfg4_wsk_$rep --solver slbfgs --steps 6 --no-cpu-baseline
LBF_NO_WSK=1 B cfg4_lds_$rep --solver slbfgs --steps 6 --no-cpu-baseline
done
B s15000_wsk --steps 400 --samples 15000 --no-cpu-baseline
echo "run d ok"
