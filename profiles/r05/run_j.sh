#!/bin/bash
# round 5, run J: the cross-process RCCL tests (two rank processes on GPU 0, NCCL_HOSTID per rank, socket
# transport on loopback) and the first-pair test split into its non-chaotic parts; then SQ counter passes
# over the 7500-row shard (the 8-rank share of cfg 2) for the forward / dW GEMMs' counter explanation.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05j
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_gpu_rccl_procs.py \
  "tests/test_gpu_fullsize.py::test_cfg4_slbfgs_first_pair_full_size" > $O/tests.log 2>&1; echo "tests rc $?"
grep -E "PASSED|FAILED|ERROR|first pair|bench --gpus" $O/tests.log | head -30
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/sq$i -o run -- python3 $R/bench.py --samples 7500 \
    --steps 5 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/sq$i.json 2> $O/sq$i.err || { echo "pmc pass $i failed"; exit 1; }
done
echo "run j ok"
