#!/bin/bash
# round 5, run AD: combine_small with its coefficients by physical ring slot (HistView::coefp, written by
# hist_core and dir_combine): every load of the lane (coefficients, live mask, every slot's values, g, x, the
# abort flag) in one round trip instead of the ring header's round trip first; tail_cols_fin's column loads go
# out with the abort flag and the ring count. Whole GPU suite, then interleaved A/B against the previous
# commit's library (ab/base, LBF_LIB_PATH).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ad
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "suite rc $rc"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernel_ms_per_step',{}); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('avg_launch_us'), d.get('final_loss',''))"; }
BASE=$R/ab/base/liblbfgs_amd_abi3.so
for rep in 1 2 3 4; do
B s7500_new_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B s7500_base_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
B c2_new_$rep --steps 400 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B c2_base_$rep --steps 400 --no-cpu-baseline || exit 1
B drv_new_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B drv_base_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
for rep in 1 2; do
B cfg4_new_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B cfg4_base_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
done
echo "run ad ok"
