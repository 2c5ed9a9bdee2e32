# A/B of the stream-ordering event scope (TPE_DEVICE_EVENTS=1 device-scope,
# 0 system-scope) on one box: GPU tests that exercise the side stream, then
# alternating bench lines (N=1 and the 8-way share) and one kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_graphs.py tests/test_gpu_suggest.py tests/test_gpu_table.py tests/test_gpu_rccl.py -m gpu > gpurun_out/ev_tests.log 2>&1 || { tail -30 gpurun_out/ev_tests.log; exit 1; }
tail -1 gpurun_out/ev_tests.log
for v in 0 1 0 1; do
  TPE_DEVICE_EVENTS=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 40 > gpurun_out/ev_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ev_$v.json'));print('events=$v N1', round(d['ms_per_step'],4), round(d['suggest_p50_ms'],4))"
done
for v in 0 1 0 1; do
  TPE_DEVICE_EVENTS=$v timeout -k 10 200 python tools/rank_share.py 8 > gpurun_out/ev_share_$v.txt 2>/dev/null || exit 1
  echo "events=$v share8: $(tail -1 gpurun_out/ev_share_$v.txt)"
done
TPE_DEVICE_EVENTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/evprof_1 -o run -- python bench.py --no-cpu-baseline --no-extras --steps 20 > /dev/null 2>&1 || exit 1
python tools/timeline.py gpurun_out/evprof_1 1
