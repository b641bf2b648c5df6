#!/bin/bash
# round 5, run T: the large-n combine with padded rounds of U = 10 pairs (m a multiple of 10) against U = 8 with
# a remainder loop (LBF_COMBINE_U8=1): the two-loop parity tests, then the n = 10.49M microbenchmark interleaved.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05t
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -2 $O/tests.log
for rep in 1 2; do
timeout -k 10 240 python -u bench_two_loop.py --m 10,20,50 > $O/u10_$rep.jsonl 2> $O/u10_$rep.err || { echo "two-loop failed"; exit 1; }
LBF_COMBINE_U8=1 timeout -k 10 240 python -u bench_two_loop.py --m 10,20,50 > $O/u8_$rep.jsonl 2> $O/u8_$rep.err || { echo "two-loop failed"; exit 1; }
for f in u10_$rep u8_$rep; do cat $O/$f.jsonl | python3 -c "import json,sys; [print('$f m', d['m'], d['roofline']['frac'], d['gram_us'], d['hist_coef_us'], d['combine_us'], d['combine_GBs']) for d in map(json.loads, sys.stdin)]"; done
done
echo "run t ok"
