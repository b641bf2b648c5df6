# Small-shard (per-rank N=7500) analysis: kernel trace + phase stamps of the optimizer tail.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
KT_N=7500 timeout -k 10 120 python -u profiles/ktrace.py > $O/ktrace_7500.txt 2>&1 && \
KT_N=60000 timeout -k 10 120 python -u profiles/ktrace.py > $O/ktrace_60000.txt 2>&1 && \
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $R/$O/prof_7500.json 2> $R/$O/prof_7500.err
echo "rc=$?"
