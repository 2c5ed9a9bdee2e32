cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r03_final_gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r03_final_bench.json 2> gpurun_out/r03_final_bench.err || exit 1
bash tools/profile_round.sh r03_final --steps 20 --warmup 3 --no-cpu-baseline --no-extras || exit 1
