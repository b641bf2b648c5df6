#!/bin/bash
# round 5, run I (re-entry after the session holding run H's results was lost): the whole GPU suite on HEAD,
# the cfg-4 full-size tests verbose (their printed deviations are the record VERDICT r04 item 1 asks for),
# smoke, the driver's shape, 400 iterations, the 7500-row shard, cfg 4 with the layer-0 forward split count
# capped at 4 and 2 (LBF_FSPLIT_CAP) beside the default; kernel traces at 7500 and cfg 4; PMC FETCH/WRITE at 7500.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05i
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "suite rc $?"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_ranks.py -k "cfg4 or slbfgs" > $O/cfg4.log 2>&1; echo "cfg4 rc $?"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'))"; }
for rep in 1 2; do
B cfg4_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_FSPLIT_CAP=4 B cfg4_fs4_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_FSPLIT_CAP=2 B cfg4_fs2_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
B s7500_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
B c2_$rep --steps 400 --no-cpu-baseline || exit 1
B drv_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
B driver --steps 20 --warmup 5 || exit 1
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/kt60000.json 2> $O/kt60000.err || { echo "prof failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc75_fetch -o run -- python3 $R/bench.py --samples 7500 --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc75_fetch.json 2> $O/pmc75_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc75_write -o run -- python3 $R/bench.py --samples 7500 --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc75_write.json 2> $O/pmc75_write.err || { echo "pmc failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv && \
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv && \
python3 profiles/kstats_live.py $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv || echo "kstats failed"
echo "run i ok"
