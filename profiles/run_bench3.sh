# cfg-5 / cfg-2 / per-rank benches (with the split plan printed) and the parity suite.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
LBF_SHOW_PLAN=1 timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 100 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 100 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/gpu_par.log 2>&1
echo "rc=$?"
grep -h "lbf plan" $O/bench_cfg5.err | sort | uniq
tail -1 $O/gpu_par.log
