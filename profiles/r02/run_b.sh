# Round 2, run B: the tests that failed in run A, after the fixes.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02b
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_dp.py tests/test_gpu_configs.py -m gpu -v -s -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -5 $O/gpu_tests.log
