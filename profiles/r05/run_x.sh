#!/bin/bash
# round 5, run X: the head tile with every LDS read of a phase issued before its MFMAs (forward, dW strips in
# interleaved pairs with dZ read once, delta over all 16-row strips at once; same chains, bitwise the same).
# The whole GPU suite; phase stamps of the fused forward GEMM (debug build of the new head, build/ktrace) at 7500 / 60000
# rows; then interleaved A/B against the previous commit's library (ab/base, LBF_LIB_PATH): the 7500-row
# shard, 400 iterations and the driver's shape of cfg 2, cfg 4.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05x
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "suite rc $rc"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
KT_RAW=$O/ktrace_blocks NS=7500,60000 timeout -k 10 200 python -u profiles/ktrace_gemm.py > $O/ktrace_gemm.txt 2>&1; echo "ktrace rc $?"; grep -v amdgpu.ids $O/ktrace_gemm.txt
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernel_ms_per_step',{}); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('final_loss',''), k.get('gemm_dw[0]'), k.get('gemm_fwd[0]'))"; }
BASE=$R/ab/base/liblbfgs_amd_abi3.so
for rep in 1 2; do
B s7500_new_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B s7500_base_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
B c2_new_$rep --steps 400 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B c2_base_$rep --steps 400 --no-cpu-baseline || exit 1
B drv_new_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B drv_base_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
B cfg4_new_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B cfg4_base_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
done
echo "run x ok"
