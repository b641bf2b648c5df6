#!/bin/bash
# round 4, run E: the S-LBFGS twin stream on a subset of the CUs (LBF_TWIN_CUS A/B) against the low-priority
# twin on all CUs.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04e
mkdir -p $O
cd $R
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; }
B cfg4_all --solver slbfgs --steps 6 --no-cpu-baseline
LBF_TWIN_CUS=64 B cfg4_cu64 --solver slbfgs --steps 6 --no-cpu-baseline
LBF_TWIN_CUS=96 B cfg4_cu96 --solver slbfgs --steps 6 --no-cpu-baseline
LBF_TWIN_CUS=128 B cfg4_cu128 --solver slbfgs --steps 6 --no-cpu-baseline
LBF_TWIN_CUS=32 B cfg4_cu32 --solver slbfgs --steps 6 --no-cpu-baseline
B cfg4_all_b --solver slbfgs --steps 6 --no-cpu-baseline
LBF_TWIN_CUS=64 B cfg4_cu64_b --solver slbfgs --steps 6 --no-cpu-baseline
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_slbfgs_run.py -x -q --timeout 200 --timeout-method thread > $O/slbfgs_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/slbfgs_tests.log; exit 1; }
tail -1 $O/slbfgs_tests.log
echo "run e ok"
