# Tuning sweep of the history sweeps at cfg-5 n: combine unroll, gram loads in flight, gram chunk.
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/sweep
mkdir -p $O
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u bench_two_loop.py --m 10,50 > $O/$name.jsonl 2> $O/$name.err
}
run base && run comb1 LBF_COMB_U=1 && run comb8 LBF_COMB_U=8 && run gram8 LBF_GRAM_U=8 && run gram16 LBF_GRAM_U=16 && \
run chunk2k LBF_GRAM_CHUNK=2048 && run chunk8k LBF_GRAM_CHUNK=8192 && run chunk2k_g8 LBF_GRAM_CHUNK=2048 LBF_GRAM_U=8
echo "rc=$?"
