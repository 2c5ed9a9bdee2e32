cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/probe_table.py 4194304 uniform,loguniform,normal table > gpurun_out/r02_quick.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r02_quick_bench.json 2>&1 || exit 1
