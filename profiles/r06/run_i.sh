#!/bin/bash
# Run I (round 6): does the Gram sweep's partial-row layout cost it? the micro-benchmark with three transposed /
# row-layout partial stores per vector, and the two-loop with LBF_GRAM_FIN=0 (row partials + fold + hist_step)
# against the default gram_fin route (transposed partials + column sums).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06i
mkdir -p $O
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 profiles/micro/ring_ld.hip -o $O/ring_ld > $O/build.txt 2>&1 || { cat $O/build.txt; exit 1; }
timeout -k 10 240 $O/ring_ld > $O/ring_ld.txt 2>&1 || { echo "ring_ld failed"; tail $O/ring_ld.txt; exit 1; }
grep -E "gram3|n = " $O/ring_ld.txt | head -12
T() { n=$1; shift; env "$@" timeout -k 10 240 python -u bench_two_loop.py --m 10,50 > $O/$n.jsonl 2> $O/$n.err || { echo "two-loop $n failed"; tail -3 $O/$n.err; exit 1; }; python3 -c "
import json
for l in open('$O/$n.jsonl'):
    d=json.loads(l); print('$n', 'm', d['m'], d['roofline']['frac'], d['gram_us'], d['hist_coef_us'], d['combine_us'], d['gram_GBs'], d['combine_GBs'])"; }
for i in 1 2; do
T fin1_$i LBF_GRAM_FIN=1
T fin0_$i LBF_GRAM_FIN=0
done
echo "run i ok"
