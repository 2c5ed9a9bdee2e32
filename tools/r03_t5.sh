cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r03_t4.sh || exit 1
timeout -k 10 60 tools/_variants/rng_microbench > gpurun_out/rng_microbench.txt 2>&1 || exit 1
bash tools/r03_issue.sh a base NO_PHILOX NO_BM NO_COMP SKIP_SCORE PHILOX_ROUNDS_7 || exit 1
