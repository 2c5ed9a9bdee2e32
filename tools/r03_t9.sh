cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_t9_new.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03_t9_bench.json 2> gpurun_out/r03_t9_bench.err || exit 1
timeout -k 10 200 python tools/probe_table.py 4194304 uniform,loguniform,normal > gpurun_out/r03_t9_probe.txt 2>&1 || exit 1
