#!/bin/bash
# round 5, run A: the cfg-4 parity record at the fixed 5 % bound (first pair after 20 SVRG steps, per-candidate
# record, world-2 epochs, replicated drift check), the CPU-baseline thread probe, then the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05a
mkdir -p $O
cd $R
timeout -k 10 90 ./profiles/micro/delivery > $O/delivery.txt 2>&1; echo "delivery rc $?"; cat $O/delivery.txt
timeout -k 10 300 python -u profiles/r05/cpu_threads.py 16 32 64 128 > $O/cpu_threads.txt 2>&1; echo "cpu probe rc $?"; cat $O/cpu_threads.txt
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py -k "cfg4" > $O/cfg4_fullsize.log 2>&1; echo "cfg4 fullsize rc $?"
grep -E "first pair|cfg4 epoch|PASS|FAIL|Error|assert" $O/cfg4_fullsize.log | head -40
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_gpu_ranks.py -k "cfg4 or drift" > $O/ranks.log 2>&1; echo "ranks rc $?"
grep -E "cfg4 epoch|PASS|FAIL|Error|assert" $O/ranks.log | head -40
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "suite rc $?"
tail -5 $O/gpu_tests.log
