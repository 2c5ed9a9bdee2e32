cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_posteriors.py tests/test_gpu_c5.py tests/test_gpu_parity.py tests/test_gpu_history.py tests/test_gpu_suggest.py > gpurun_out/r02_fit_tests.log 2>&1 || exit 1
timeout -k 10 400 python tools/rank_share.py 8 > gpurun_out/r02_rank_share.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r02share; mkdir -p gpurun_out/prof_r02share
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02share/trace -o run -- python3 tools/rank_share.py --only 8 2 > gpurun_out/prof_r02share/trace.log 2>&1
