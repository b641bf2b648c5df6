#!/bin/bash
# Run K (round 6): the ring-stride micro-benchmark with the Gram sweep's first phase (gram3p_k): does forming s, y, g cost the engine's sweep its last 10 %?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06k
mkdir -p $O
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 profiles/micro/ring_ld.hip -o $O/ring_ld > $O/build.txt 2>&1 || { cat $O/build.txt; exit 1; }
timeout -k 10 240 $O/ring_ld > $O/ring_ld.txt 2>&1 || { echo "ring_ld failed"; tail $O/ring_ld.txt; exit 1; }
cat $O/ring_ld.txt
