cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r02_quick_bench.json 2>&1 || exit 1
timeout -k 10 600 python tools/rank_share.py 8 > gpurun_out/r02_rank_share.txt 2>&1 || exit 1
