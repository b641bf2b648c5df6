#!/bin/bash
# round 5, run G: cfg-4 parity (first pair at the device's own FD points, ReLU epoch, tanh epoch), the whole
# GPU suite, then A/B of the round's kernel changes: the wave-split-K 32 x 128 GEMM (LBF_NO_WSK=1 for the LDS-DMA
# loop) and the compact-form two-loop coefficients (LBF_NO_COMPACT=1 for the recurrences), interleaved
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py -k "cfg4" > $O/cfg4.log 2>&1; echo "cfg4 rc $?"
grep -E "first pair|cfg4 |PASSED|FAILED|Error" $O/cfg4.log | head -30
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "suite rc $?"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('kernel_ms_per_step'))"; }
for rep in 1 2; do
B s7500_new_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_NO_WSK=1 B s7500_nowsk_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_NO_COMPACT=1 B s7500_nocompact_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
done
for rep in 1 2; do
B cfg4_new_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_NO_WSK=1 B cfg4_nowsk_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_NO_COMPACT=1 B cfg4_nocompact_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
done
for rep in 1 2; do
B c2_new_$rep --steps 400 --no-cpu-baseline || exit 1
LBF_NO_COMPACT=1 B c2_nocompact_$rep --steps 400 --no-cpu-baseline || exit 1
done
B driver --steps 20 --warmup 5 || exit 1
echo "run g ok"
