#!/bin/bash
# Run E (round 6): the stream-K A/B of run C without the test suite (run C: 314 passed, 1 Armijo-trajectory bound).
# against LBF_FWD_SK=0 (cfg 2 driver shape and 400 iterations, cfg 3), and a kernel trace of cfg 2 with it.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06e
mkdir -p $O
cd $R
echo "tests skipped (run C)"
tail -1 $O/gpu_tests.log
B() { n=$1; shift; timeout -k 10 240 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('evals_per_iter'))"; }
for i in 1 2; do
LBF_FWD_SK=1 B sk1_400_$i --steps 400 --no-cpu-baseline
LBF_FWD_SK=0 B sk0_400_$i --steps 400 --no-cpu-baseline
LBF_FWD_SK=1 B sk1_drv_$i --steps 20 --warmup 5 --no-cpu-baseline
LBF_FWD_SK=0 B sk0_drv_$i --steps 20 --warmup 5 --no-cpu-baseline
done
LBF_FWD_SK=1 B sk1_cfg3 --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline
LBF_FWD_SK=0 B sk0_cfg3 --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 100 --warmup 5 > $O/kt60000.json 2> $O/kt60000.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv || echo "kstats failed"
head -4 $O/kt60000_live.csv
echo "run c ok"
