cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sorted_fit.py tests/test_gpu_history.py tests/test_gpu_replay.py tests/test_gpu_lattice.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_t6_new.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03_t6_bench.json 2> gpurun_out/r03_t6_bench.err || exit 1
bash tools/profile_round.sh r03_d --steps 20 --warmup 3 --no-cpu-baseline --no-extras
