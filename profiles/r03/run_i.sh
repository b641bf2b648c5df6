# Round 3, run I: the periodic pair of ~6 us gaps every 5 iterations (25 launches) at 7500 rows: does the
# HIP kernel-argument placement change it (HIP_FORCE_DEV_KERNARG 0/1)?
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03i
mkdir -p $O
cd /tmp
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k LBF_HOST_TIMING=1 timeout -k 10 120 python3 $R/bench.py --samples 7500 --no-cpu-baseline > $O/bench_k$k.json 2> $O/bench_k$k.err || exit 1
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_k$k -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt_k$k.json 2> $O/kt_k$k.err || exit 1
done
echo "rc=$?"
