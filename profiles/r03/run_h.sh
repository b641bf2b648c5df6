# Round 3, run H: the stream query in the speculative loop's wait only after 5 ms of spinning (it enqueued
# a marker per iteration); 7500 / 60000-row benches with host timing, kernel trace + gaps at 7500.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03h
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "spec or fused or tail" > $O/tail_tests.log 2>&1 || { echo "tail tests failed"; tail -5 $O/tail_tests.log; exit 1; }
tail -1 $O/tail_tests.log
cd /tmp
for n in 7500 60000; do
  LBF_HOST_TIMING=1 timeout -k 10 120 python3 $R/bench.py --samples $n --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err || exit 1
cd $R
python3 profiles/gaps.py $O/kt7500/run_kernel_trace.csv > $O/gaps.txt
echo "rc=$?"
