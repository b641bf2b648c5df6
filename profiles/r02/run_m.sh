# Round 2, run M: dW tile at the shard sizes (64 x 64 default below 16k rows vs 128 x 128: LBF_DW_TILE64=0),
# interleaved, plus the DP route (1-rank communicator) at 7500 / 15000 / 30000 rows.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02m
mkdir -p $O
cd $R
for rep in 1 2; do
  for S in 7500 15000; do
    timeout -k 10 120 python -u bench.py --samples $S --no-cpu-baseline --steps 300 > $O/s${S}_d64_$rep.json 2> $O/s${S}_d64_$rep.err || exit 1
    LBF_DW_TILE64=0 timeout -k 10 120 python -u bench.py --samples $S --no-cpu-baseline --steps 300 > $O/s${S}_d128_$rep.json 2> $O/s${S}_d128_$rep.err || exit 1
  done
done
for S in 7500 15000 30000; do
  timeout -k 10 120 python -u bench.py --samples $S --no-cpu-baseline --comm1 > $O/s${S}_comm1.json 2> $O/s${S}_comm1.err || exit 1
done
echo "rc=0"
