# round-2 profiles: bench trace + PMC passes, then a C4 kernel trace
set -e
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r02a --steps 3 --warmup 1 --no-cpu-baseline --no-extras
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r02c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02c4/trace -o run -- python3 tools/scale_configs.py c4 > gpurun_out/prof_r02c4/trace.log 2>&1
echo ok
