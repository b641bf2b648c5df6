#!/bin/bash
# Run A (round 6): the new parity tests (teacher-forced S-LBFGS epochs, the K-map route, cfg 5 at 8192 rows,
# the cross-process RCCL tests with the polling runner), then the cfg-5 plan print.
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ranks.py tests/test_gpu_fullsize.py \
  tests/test_gpu_rccl_procs.py -k "kmat_route or split_plan or forced or cfg4 or rccl or bench_two" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -50 $O/tests.log; exit 1; }
tail -5 $O/tests.log
LBF_SHOW_PLAN=1 timeout -k 10 120 python -u profiles/r06/show_plan_cfg5.py > $O/plan_cfg5.txt 2>&1
echo "plan rc=$?"
