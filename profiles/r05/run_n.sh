#!/bin/bash
# round 5, run N: the epoch-end full-batch evaluation ahead on a third stream (SlbfgsSolver::post_full). The
# whole GPU suite; cfg 4 against LBF_NO_FULL_AHEAD=1, interleaved; the wave-split-K GEMM (LBF_WSK=1) against
# the LDS-DMA loop again at the 7500-row shard, now that the 32-row head tile runs half its steps.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05n
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "suite rc $rc"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernel_ms_per_step',{}); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('final_loss',''), k.get('gemm_dw[0]'), k.get('gemm_fwd[0]'))"; }
for rep in 1 2 3; do
B cfg4_new_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_NO_FULL_AHEAD=1 B cfg4_base_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
done
for rep in 1 2; do
B s7500_lds_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_WSK=1 B s7500_wsk_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
done
echo "run n ok"
