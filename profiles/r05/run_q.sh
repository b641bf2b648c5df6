#!/bin/bash
# round 5, run Q: PMC FETCH/WRITE (cfg 2 driver shape, cfg 4) for the bench lines' traffic field, and the forward
# GEMM's per-block stamps with placement (debug build build/ktrace, raw per-block CSV). Run P's PMC passes
# stopped at a bench.py KeyError (the breakdown's dominant section under counter serialisation was one that
# runs only at the solve's start; fixed: the dominant section is chosen among those run every iteration).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05q
mkdir -p $O
cd /tmp
for m in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc60_$m -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc60_$m.json 2> $O/pmc60_$m.err || { echo "pmc60 $m failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc4_$m -o run -- python3 $R/bench.py --solver slbfgs --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc4_$m.json 2> $O/pmc4_$m.err || { echo "pmc4 $m failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $O/pmc75_$m -o run -- python3 $R/bench.py --samples 7500 --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/pmc75_$m.json 2> $O/pmc75_$m.err || { echo "pmc75 $m failed"; exit 1; }
done
cd $R
KT_RAW=$O/ktrace_blocks NS=7500,60000 timeout -k 10 200 python -u profiles/ktrace_gemm.py > $O/ktrace_gemm.txt 2>&1; echo "ktrace rc $?"
grep -v amdgpu.ids $O/ktrace_gemm.txt | tail -8
echo "run q ok"
