cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pruned64.py > gpurun_out/r02_p64_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_pruned64.py > gpurun_out/r02_p64.txt 2>&1 || exit 1
timeout -k 10 300 python tools/profile_c4.py 256 > gpurun_out/r02_c4_prof.txt 2>&1 || exit 1
