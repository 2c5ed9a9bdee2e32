cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_table.py tests/test_gpu_c5.py tests/test_gpu_parity.py tests/test_gpu_c4.py > gpurun_out/r02_build_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r02_quick_bench.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r02d; mkdir -p gpurun_out/prof_r02d
TPE_SIDE_STREAM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02d/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_r02d/trace.log 2>&1
