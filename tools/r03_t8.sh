cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_c5.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_t8_new.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03_t8_bench.json 2> gpurun_out/r03_t8_bench.err || exit 1
timeout -k 10 200 python tools/probe_table.py 4194304 uniform,loguniform,normal > gpurun_out/r03_t8_probe.txt 2>&1 || exit 1
timeout -k 10 400 python tools/rank_share.py 2 4 8 > gpurun_out/r03_t8_rank_share.txt 2>&1 || exit 1
