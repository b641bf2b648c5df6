#!/bin/bash
# round 5, run Z: the wave-split-K direct-load 32 x 128 forward (LBF_WSK=1) against the LDS-DMA loop at the
# 7500-row shard, by kernel time (rocprofv3 kernel trace, live launches) rather than iterations/s, twice each,
# interleaved; then the bench lines.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05z
mkdir -p $O
cd /tmp
for rep in 1 2; do
for v in lds wsk; do
  if [ $v = wsk ]; then export LBF_WSK=1; else unset LBF_WSK; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${v}_$rep -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 200 > $O/kt_${v}_$rep.json 2> $O/kt_${v}_$rep.err || { echo "prof $v failed"; tail -3 $O/kt_${v}_$rep.err; exit 1; }
  python3 $R/profiles/kstats_live.py --spec $O/kt_${v}_$rep/run_kernel_trace.csv --out $O/kt_${v}_${rep}_live.csv > /dev/null && head -4 $O/kt_${v}_${rep}_live.csv | cut -c1-150
  tail -1 $O/kt_${v}_$rep.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rep', d['value'], d['ms_per_step'])"
done
done
unset LBF_WSK
cd $R
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('avg_launch_us'))"; }
for rep in 1 2 3; do
B s7500_lds_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_WSK=1 B s7500_wsk_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
done
echo "run z ok"
