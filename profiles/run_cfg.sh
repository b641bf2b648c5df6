# BASELINE configs 3-5 parity tests, then a config-5 bench (1 GPU, N = 1M, m = 50).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $O/gpu_cfg.log 2>&1 && \
timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --cpu-iters 2 --cpu-samples 400 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
echo "rc=$?"
