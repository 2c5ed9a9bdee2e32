# Prefix-first lattice argmax (tpe_lattice_suggest): GPU tests, then an A/B
# against full streams (TPE_LAT_PREFIX=0) on one box and one kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lattice.py tests/test_gpu_graphs.py tests/test_gpu_suggest.py tests/test_gpu_plan_cache.py tests/test_gpu_history.py tests/test_gpu_rccl.py -m gpu > gpurun_out/lat_tests.log 2>&1 || { tail -40 gpurun_out/lat_tests.log; exit 1; }
tail -1 gpurun_out/lat_tests.log
for v in 0 65536 0 65536; do
  TPE_LAT_PREFIX=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 40 > gpurun_out/lat_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lat_$v.json'));print('prefix=$v N1', round(d['ms_per_step'],4), round(d['suggest_p50_ms'],4))"
done
for v in 0 65536; do
  TPE_LAT_PREFIX=$v timeout -k 10 200 python tools/rank_share.py 8 > gpurun_out/lat_share_$v.txt 2>/dev/null || exit 1
  echo "prefix=$v share8: $(tail -1 gpurun_out/lat_share_$v.txt)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/latprof -o run -- python bench.py --no-cpu-baseline --no-extras --steps 20 > /dev/null 2>&1 || exit 1
python tools/timeline.py gpurun_out/latprof 1
