cd $GRAFT_REPO_ROOT
out=gpurun_out/r02_side.txt
: > $out
for m in 0 1 2; do
  echo "== TPE_SIDE_STREAM=$m" >> $out
  TPE_SIDE_STREAM=$m timeout -k 10 300 python tools/rank_share.py 8 2>/dev/null | grep -v amdgpu >> $out || exit 1
done
TPE_SIDE_STREAM=1 timeout -k 10 300 python -m pytest -q -x --timeout 120 tests/test_gpu_parity.py tests/test_gpu_suggest.py tests/test_gpu_history.py 2>&1 | tail -2 >> $out
