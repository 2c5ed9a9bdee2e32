cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/profile_c4.py 512 > gpurun_out/r02_c4side_1.txt 2>&1 || exit 1
TPE_SIDE_STREAM=0 timeout -k 10 300 python tools/profile_c4.py 512 > gpurun_out/r02_c4side_0.txt 2>&1 || exit 1
