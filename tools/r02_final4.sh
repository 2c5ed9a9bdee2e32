# round-2 final validation (GPU box), after the prefix-first lattice path and the table-build reductions:
# full GPU suite, smoke, bench, configs, rank shares, kernel trace + PMC
# passes, an 8-way share kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/full.log 2>&1 || { tail -30 gpurun_out/full.log; exit 1; }
tail -1 gpurun_out/full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python tools/scale_configs.py > gpurun_out/configs.json 2> gpurun_out/configs.err || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python tools/rank_share.py 2 4 8 > gpurun_out/rs_final.txt 2>&1 || exit 1
bash tools/profile_round.sh r02_j > gpurun_out/prof_r02_j.log 2>&1 || exit 1
mkdir -p gpurun_out/prof_r02jshare
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02jshare/trace -o run -- python3 tools/rank_share.py --only 8 2 > gpurun_out/prof_r02jshare/trace.log 2>&1 || exit 1
echo ok
