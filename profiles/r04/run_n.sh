#!/bin/bash
# round 4, run N: cfg 4 timing diagnostics: the inner-step chain alone (LBF_DIAG_ANCHOR=1, anchor gradients
# zero: wrong results, timing only), the anchor gradient serial on the context stream (=2), the twin (default)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04n
mkdir -p $O
cd $R
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step'))"; }
B twin_a --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DIAG_ANCHOR=1 B alone_a --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DIAG_ANCHOR=2 B serial_a --solver slbfgs --steps 6 --no-cpu-baseline
B twin_b --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DIAG_ANCHOR=1 B alone_b --solver slbfgs --steps 6 --no-cpu-baseline
LBF_DIAG_ANCHOR=2 B serial_b --solver slbfgs --steps 6 --no-cpu-baseline
cd /tmp
export LBF_DIAG_ANCHOR=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4_alone -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4_alone.json 2> $O/kt4_alone.err || { echo "prof failed"; exit 1; }
export LBF_DIAG_ANCHOR=2
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4_serial -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4_serial.json 2> $O/kt4_serial.err || { echo "prof failed"; exit 1; }
unset LBF_DIAG_ANCHOR
cd $R
python3 profiles/kstats_live.py $O/kt4_alone/run_kernel_trace.csv --out $O/kt4_alone_live.csv && \
python3 profiles/kstats_live.py $O/kt4_serial/run_kernel_trace.csv --out $O/kt4_serial_live.csv || { echo "kstats failed"; exit 1; }
echo "run n ok"
