cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cat_prefix.py tests/test_gpu_table.py tests/test_gpu_c5.py tests/test_gpu_sorted_fit.py tests/test_gpu_history.py tests/test_gpu_lattice.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_t4_new.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03_t4_bench.json 2> gpurun_out/r03_t4_bench.err || exit 1
timeout -k 10 200 python tools/probe_table.py 4194304 uniform,loguniform,normal > gpurun_out/r03_t4_probe.txt 2>&1 || exit 1
