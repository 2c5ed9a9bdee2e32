cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_c5.py tests/test_gpu_sorted_fit.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r03_t3_new.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r03_t3_bench.json 2> gpurun_out/r03_t3_bench.err || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_t3_gpu_tests.log 2>&1 || exit 1
bash tools/profile_round.sh r03_b --steps 20 --warmup 3 --no-cpu-baseline --no-extras
