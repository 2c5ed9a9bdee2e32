cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/scale_configs.py c2 c5 c4 > gpurun_out/r02_configs.json 2> gpurun_out/r02_configs.err || exit 1
