#!/bin/bash
# round 4, run Q: why the DP code path (1-rank RCCL communicator) costs 35 us per iteration at 7500 rows:
# kernel traces of --comm1 and the single route, idle gaps per kernel (profiles/gaps.py)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q
mkdir -p $O
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_comm1 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 100 --device-warmup 0 --comm1 > $O/kt_comm1.json 2> $O/kt_comm1.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_single -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 100 --device-warmup 0 > $O/kt_single.json 2> $O/kt_single.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/gaps.py $O/kt_comm1/run_kernel_trace.csv --tail 700 > $O/gaps_comm1.txt && \
python3 profiles/gaps.py $O/kt_single/run_kernel_trace.csv --tail 540 > $O/gaps_single.txt || { echo "gaps failed"; exit 1; }
cat $O/gaps_comm1.txt $O/gaps_single.txt
python3 profiles/kstats_live.py --spec $O/kt_comm1/run_kernel_trace.csv --out $O/kt_comm1_live.csv || echo "kstats failed"
echo "run q ok"
