#!/bin/bash
# Round-4 final evidence on the GPU box: the bench line, the kernel-trace
# summary + PMC passes (tools/profile_round.sh), and the rank-share projection.
cd $GRAFT_REPO_ROOT
TAG=${1:-r04_final}
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
tail -c 600 gpurun_out/${TAG}_bench.json
bash tools/profile_round.sh $TAG --steps 20 --warmup 3 --no-cpu-baseline --no-extras || exit 1
timeout -k 10 400 python -u tools/rank_share.py 2 4 8 > gpurun_out/${TAG}_rank_share.txt 2>&1 || exit 1
tail -4 gpurun_out/${TAG}_rank_share.txt
