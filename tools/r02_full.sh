cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_lattice_diag.py > gpurun_out/r02_lat.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --no-extras > gpurun_out/r02_quick_bench.json 2>&1 || exit 1
