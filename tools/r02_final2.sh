cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || exit 1
timeout -k 10 600 python tools/scale_configs.py c2 c5 c4 > gpurun_out/r02_configs.json 2> gpurun_out/r02_configs.err || exit 1
timeout -k 10 600 python tools/rank_share.py 2 4 8 > gpurun_out/r02_rank_share.txt 2>&1 || exit 1
bash tools/profile_round.sh r02e --steps 3 --warmup 1 --no-cpu-baseline --no-extras || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r02f
TPE_SIDE_STREAM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02f/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_r02f/trace.log 2>&1
