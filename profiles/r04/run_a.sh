#!/bin/bash
# round 4: GPU suite + smoke + benches on the current tree (pruned routes, ABI 3)
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 120 python bench.py --steps 400 --no-cpu-baseline > $O/bench_400.json 2> $O/bench_400.err &&
LBF_DW_K2=0 timeout -k 10 120 python bench.py --steps 400 --no-cpu-baseline > $O/bench_400_nok2.json 2> $O/bench_400_nok2.err &&
timeout -k 10 120 python bench.py --steps 400 --no-cpu-baseline > $O/bench_400_b.json 2> $O/bench_400_b.err &&
timeout -k 10 120 python bench.py --steps 400 --samples 7500 --no-cpu-baseline > $O/bench_7500.json 2> $O/bench_7500.err &&
timeout -k 10 180 python bench.py --solver slbfgs --steps 6 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err &&
LBF_ROWHEAD=0 timeout -k 10 180 python bench.py --solver slbfgs --steps 6 --no-cpu-baseline > $O/bench_cfg4_norowhead.json 2> $O/bench_cfg4_norowhead.err &&
timeout -k 10 180 python bench.py --solver slbfgs --steps 6 --no-cpu-baseline --comm1 > $O/bench_cfg4_comm1_repl.json 2> $O/bench_cfg4_comm1_repl.err &&
timeout -k 10 120 python profiles/r04/cfg4_fullbatch.py > $O/cfg4_fullbatch.json 2> $O/cfg4_fullbatch.err &&
timeout -k 10 120 ./profiles/micro/launch_floor > $O/launch_floor.txt 2>&1 &&
timeout -k 10 300 python bench_two_loop.py > $O/two_loop.jsonl 2> $O/two_loop.err
