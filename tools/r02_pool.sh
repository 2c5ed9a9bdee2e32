cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sampler.py tests/test_gpu_lattice.py tests/test_gpu_table.py tests/test_gpu_shard.py > gpurun_out/r02_pool_tests.log 2>&1 || exit 1
bash tools/r02_var_table.sh
