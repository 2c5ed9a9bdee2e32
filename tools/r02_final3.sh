# round-2 final validation (GPU box): full GPU suite, smoke, bench, configs, profiles
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/full.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python tools/scale_configs.py > gpurun_out/configs.json 2> gpurun_out/configs.err || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python tools/rank_share.py 2 4 8 > gpurun_out/rs_final.txt 2>&1 || exit 1
