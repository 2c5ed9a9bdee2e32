cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r03_final2_bench.json 2> gpurun_out/r03_final2_bench.err || exit 1
bash tools/profile_round.sh r03_final2 --steps 20 --warmup 3 --no-cpu-baseline --no-extras || exit 1
timeout -k 10 400 python tools/rank_share.py 2 4 8 > gpurun_out/r03_final2_rank_share.txt 2>&1 || exit 1
