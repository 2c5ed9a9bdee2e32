cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r02c
TPE_SIDE_STREAM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02c/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_r02c/trace.log 2>&1
