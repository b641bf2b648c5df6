#!/bin/bash
# round 5, run L: phase stamps of the fused forward GEMM + head (debug build build/ktrace, LBF_KTRACE) at
# 7500 and 60000 rows; then the release build with the XCD placement on the dW GEMMs only: cfg 4 and the
# 7500-row shard against LBF_NO_XCD=1, interleaved.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05l
mkdir -p $O
cd $R
NS=7500,60000 timeout -k 10 200 python -u profiles/ktrace_gemm.py > $O/ktrace_gemm.txt 2>&1; echo "ktrace rc $?"; cat $O/ktrace_gemm.txt | grep -v amdgpu.ids
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('final_loss',''), d.get('kernel_ms_per_step',{}).get('gemm_dw[0]'), d.get('kernel_ms_per_step',{}).get('gemm_fwd[0]'))"; }
for rep in 1 2; do
B cfg4_xcd_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_NO_XCD=1 B cfg4_base_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
B s7500_xcd_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_NO_XCD=1 B s7500_base_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
done
echo "run l ok"
