cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_base_gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r03_base_bench.json 2> gpurun_out/r03_base_bench.err || exit 1
