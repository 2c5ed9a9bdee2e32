cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_r02c4b; mkdir -p gpurun_out/prof_r02c4b
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02c4b/trace -o run -- python3 tools/scale_configs.py c4 > gpurun_out/prof_r02c4b/trace.log 2>&1
