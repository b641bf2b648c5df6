#!/bin/bash
# round 5, run S: two GEMM main-loop changes. (1) quad-pipelined fragment reads (each quad of k-steps' LDS reads
# issued before the previous quad's MFMAs, quad 0 before the DMA issue) in every LDS-DMA GEMM; (2) the 32 x 128
# tile's loop with two k-tiles per barrier (PAIR, six stages). The whole GPU suite on both; interleaved A/B:
# (1) against the library built with -DLBF_NO_QPIPE (ab/noqpipe, LBF_LIB_PATH) at cfg 2 (400 iterations and the
# driver's shape), the 7500-row shard and cfg 4; (2) against LBF_NO_PAIR=1 at 7500 rows, cfg 4, cfg 3.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "suite rc $rc"; tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B() { n=$1; shift 1; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; return 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernel_ms_per_step',{}); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('final_loss',''), k.get('gemm_fwd[0]'), k.get('gemm_dw[0]'), k.get('gemm_dx[1]'))"; }
NQ=$R/ab/noqpipe/liblbfgs_amd_abi3.so
for rep in 1 2; do
B c2_q_$rep --steps 400 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$NQ B c2_nq_$rep --steps 400 --no-cpu-baseline || exit 1
B drv_q_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$NQ B drv_nq_$rep --steps 20 --warmup 5 --no-cpu-baseline || exit 1
B s7500_q_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$NQ B s7500_nq_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
LBF_NO_PAIR=1 B s7500_nopair_$rep --steps 400 --samples 7500 --no-cpu-baseline || exit 1
B cfg4_q_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_LIB_PATH=$NQ B cfg4_nq_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
LBF_NO_PAIR=1 B cfg4_nopair_$rep --solver slbfgs --steps 6 --no-cpu-baseline || exit 1
B cfg3_q_$rep --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline || exit 1
LBF_NO_PAIR=1 B cfg3_nopair_$rep --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline || exit 1
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err || echo "prof failed"
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv && head -3 $O/kt60000_live.csv
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv && head -3 $O/kt7500_live.csv
echo "run s ok"
