# A/B of library variants (build dirs given as arguments) on the cfg-2 bench: gemm_fwd[0] launch time
# (roofline avg_launch_us) and iterations/s, plus correctness of each variant (loss/grad vs the oracle).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02exp
mkdir -p $O
cd $R
for v in "$@"; do
  n=$(echo $v | tr '/' '_')
  LBF_LIB_PATH=$R/lbfgs-ffnn_amd/$v/liblbfgs_amd.so timeout -k 10 120 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_fold.py -q -x --timeout 120 --timeout-method thread -k "loss_grad or fold" > $O/t_$n.log 2>&1 || { echo "tests failed for $v"; tail -5 $O/t_$n.log; exit 1; }
  for rep in 1 2; do
    LBF_LIB_PATH=$R/lbfgs-ffnn_amd/$v/liblbfgs_amd.so timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || exit 1
  done
done
python3 - "$@" <<'PY'
import json, sys, os
O = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", "r02exp")
for v in sys.argv[1:]:
    n = v.replace("/", "_")
    for rep in (1, 2):
        d = json.load(open(f"{O}/b_{n}_{rep}.json"))
        print(f"{v:14s} rep{rep} it/s {d['value']:8.1f} evals/it {d['evals_per_iter']} fwd {d['roofline']['avg_launch_us']} us "
              f"kms {d['kernel_ms_per_step']}")
PY
