#!/bin/bash
# Run G (round 6): the ring-stride micro-benchmark with the Gram sweep's own arithmetic (three fp64 dots per history
# vector, gram3_k): is the Gram kernel's 5.4 TB/s its arithmetic or its pattern?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 profiles/micro/ring_ld.hip -o $O/ring_ld > $O/build.txt 2>&1 || { cat $O/build.txt; exit 1; }
timeout -k 10 240 $O/ring_ld > $O/ring_ld.txt 2>&1 || { echo "ring_ld failed"; tail $O/ring_ld.txt; exit 1; }
cat $O/ring_ld.txt
