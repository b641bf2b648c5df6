#!/bin/bash
# round 5, run AF: two header-dependent round trips off the S-LBFGS inner step: dir_combine stages the
# coefficient map K for 2m rows and columns (no live count first) and dir_cols issues its column loads with
# the live count. The whole GPU suite, then cfg 4 interleaved against the previous commit's library (ab/base,
# LBF_LIB_PATH), and the 7500-row shard once each (dir kernels are not on that path).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05af
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "suite rc $rc"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('avg_launch_us'), d.get('final_loss',''))"; }
BASE=$R/ab/base/liblbfgs_amd_abi3.so
for rep in 1 2 3 4; do
B cfg4_new_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B cfg4_base_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
done
B s7500_new --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$BASE B s7500_base --steps 400 --samples 7500 --no-cpu-baseline || exit 1
echo "run af ok"
