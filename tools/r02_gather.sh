cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_history.py tests/test_gpu_c4.py tests/test_gpu_suggest.py tests/test_gpu_c5.py > gpurun_out/r02_gather_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r02_quick_bench.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r02share; mkdir -p gpurun_out/prof_r02share
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02share/trace -o run -- python3 tools/rank_share.py --only 8 2 > gpurun_out/prof_r02share/trace.log 2>&1
