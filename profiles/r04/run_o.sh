#!/bin/bash
# round 4, run O: the S-LBFGS minibatch dX GEMM (256 x 512, K = 256) on 64 x 64 / 64 x 128 tiles against
# 32 x 128 (LBF_DX_TILE A/B), parity first
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04o
mkdir -p $O
cd $R
LBF_DX_TILE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_dx2.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_dx2.log; exit 1; }
tail -1 $O/gpu_tests_dx2.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step',{}).get('gemm_dx[1]'))"; }
B base_a --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DX_TILE=2 B dx64_a --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DX_TILE=3 B dx64x128_a --solver slbfgs --steps 6 --no-cpu-baseline
B base_b --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DX_TILE=2 B dx64_b --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DX_TILE=3 B dx64x128_b --solver slbfgs --steps 6 --no-cpu-baseline
echo "run o ok"
