# Round 3, run F: where does the ~6 us gap in front of combine_small come from (tail split / speculation depth
# A/B on the 7500-row shard); launch floor incl. the cross-stream hand-off costs; the two-loop microbench
# with 4 / 8 history loads in flight per lane (LBF_GRAM_U); tail_reduce back on its LDS dot phase.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03f
mkdir -p $O
cd $R
timeout -k 10 90 ./profiles/micro/launch_floor > $O/launch_floor.txt 2>&1 || echo "launch_floor failed"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "spec or fused or tail" > $O/tail_tests.log 2>&1 || { echo "tail tests failed"; tail -5 $O/tail_tests.log; exit 1; }
tail -1 $O/tail_tests.log
cd /tmp
for v in base split depth8; do
  case $v in base) E="";; split) E="LBF_TAIL_SPLIT=1";; depth8) E="LBF_SPEC_DEPTH=8";; esac
  env $E timeout -k 10 120 python3 $R/bench.py --samples 7500 --no-cpu-baseline > $O/bench_7500_$v.json 2> $O/bench_7500_$v.err || exit 1
done
LBF_TAIL_SPLIT=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt7500_split -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500_split.json 2> $O/kt7500_split.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err || exit 1
cd $R
python3 profiles/gaps.py $O/kt7500_split/run_kernel_trace.csv > $O/gaps_split.txt
python3 profiles/gaps.py $O/kt7500/run_kernel_trace.csv > $O/gaps_base.txt
timeout -k 10 200 python -u bench_two_loop.py --m 10,50 > $O/two_loop_u4.jsonl 2> $O/two_loop_u4.err && \
LBF_GRAM_U=8 timeout -k 10 200 python -u bench_two_loop.py --m 10,50 > $O/two_loop_u8.jsonl 2> $O/two_loop_u8.err
echo "rc=$?"
