#!/bin/bash
# round 5, run K: XCD-aware placement of the split-K GEMMs (gemm.hip xcd_tile). The whole GPU suite on it,
# then interleaved A/B against LBF_NO_XCD=1 (the previous placement) at the 7500-row shard, the driver's
# shape, 400 iterations of cfg 2 and cfg 4; PMC FETCH/WRITE at 7500 rows and cfg 4 with the new placement.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "suite rc $rc"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('final_loss',''), d.get('kernel_ms_per_step',{}).get('gemm_dw[0]'), d.get('kernel_ms_per_step',{}).get('gemm_fwd[0]'))"; }
for rep in 1 2; do
B s7500_xcd_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_NO_XCD=1 B s7500_base_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
B cfg4_xcd_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_NO_XCD=1 B cfg4_base_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
B c2_xcd_$rep --steps 400 --no-cpu-baseline || exit 1
LBF_NO_XCD=1 B c2_base_$rep --steps 400 --no-cpu-baseline || exit 1
B drv_xcd_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
LBF_NO_XCD=1 B drv_base_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
cd /tmp
for m in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc75_$m -o run -- python3 $R/bench.py --samples 7500 --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc75_$m.json 2> $O/pmc75_$m.err || { echo "pmc failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc4_$m -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc4_$m.json 2> $O/pmc4_$m.err || { echo "pmc failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc60_$m -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc60_$m.json 2> $O/pmc60_$m.err || { echo "pmc failed"; exit 1; }
done
echo "run k ok"
