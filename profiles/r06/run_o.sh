#!/bin/bash
# Run O (round 6): the chunked combine's vectors and quads per lane in flight (LBF_COMBINE_VQ = V Q: 24 default, 14, 22, 42), two-loop m = 10 / 20 / 50.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06o
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
T() { n=$1; shift; env "$@" timeout -k 10 300 python -u bench_two_loop.py --m 10,20,50 > $O/$n.jsonl 2> $O/$n.err || { echo "two-loop $n failed"; tail -3 $O/$n.err; exit 1; }; python3 -c "
import json
for l in open('$O/$n.jsonl'):
    d=json.loads(l); print('$n', 'm', d['m'], d['roofline']['frac'], d['gram_us'], d['hist_coef_us'], d['combine_us'], d['gram_GBs'], d['combine_GBs'])"; }
for i in 1 2; do
for v in 24 14 22 42; do
T vq${v}_$i LBF_COMBINE_VQ=$v
done
done
echo "run o ok"
