cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || exit 1
timeout -k 10 600 python tools/scale_configs.py c2 c5 c4 > gpurun_out/r02_configs.json 2> gpurun_out/r02_configs.err || exit 1
