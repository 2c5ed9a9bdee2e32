cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r02share
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02share/trace -o run -- python3 tools/rank_share.py --only 8 2 > gpurun_out/prof_r02share/trace.log 2>&1
