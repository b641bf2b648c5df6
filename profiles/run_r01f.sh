export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 240 python -u bench_two_loop.py > $O/two_loop.jsonl 2> $O/two_loop.err && \
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_tl -o run -- python3 $R/bench_two_loop.py --m 50 > $R/$O/two_loop_prof.jsonl 2> $R/$O/two_loop_prof.err
echo "rc=$?"
