cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c4.py tests/test_gpu_suggest.py > gpurun_out/r02_c4_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/profile_c4.py 256 > gpurun_out/r02_c4_prof.txt 2>&1 || exit 1
timeout -k 10 400 python tools/scale_configs.py c4 > gpurun_out/r02_c4.json 2> gpurun_out/r02_c4.err || exit 1
