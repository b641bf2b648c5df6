#!/bin/bash
# Run N (round 6): the two-loop on the round's history route (chunked combine; split Gram sweep and fold route for
# m >= 20 / > 20; gram_fin with row-major partials for m <= 20) against round 5's (LBF_COMBINE_CHUNK=0
# LBF_GRAM_SPLIT=0 LBF_GRAM_FIN=1 LBF_GRAM_ROUNDS=1), interleaved, after the parity files.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06n
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
T() { n=$1; shift; env "$@" timeout -k 10 300 python -u bench_two_loop.py --m 10,20,50 > $O/$n.jsonl 2> $O/$n.err || { echo "two-loop $n failed"; tail -3 $O/$n.err; exit 1; }; python3 -c "
import json
for l in open('$O/$n.jsonl'):
    d=json.loads(l); print('$n', 'm', d['m'], d['roofline']['frac'], d['gram_us'], d['hist_coef_us'], d['combine_us'], d['gram_GBs'], d['combine_GBs'])"; }
for i in 1 2; do
T new_$i LBF_NONE=1
T r05_$i LBF_COMBINE_CHUNK=0 LBF_GRAM_SPLIT=0 LBF_GRAM_FIN=1 LBF_GRAM_ROUNDS=1
done
echo "run n ok"
