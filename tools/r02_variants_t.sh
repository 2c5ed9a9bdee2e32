# bench group times + table tests for each tools/_variants/lib_*.so (and the in-tree lib)
cd $GRAFT_REPO_ROOT
out=gpurun_out/r02_variants.txt
: > $out
for f in "" tools/_variants/lib_*.so; do
  echo "== ${f:-base}" >> $out
  lib=${f:+$PWD/$f}
  HYPEROPT_AMD_LIB=${lib:-$PWD/hyperopt_amd/libtpe_hip.so} timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['group_ms'])" >> $out || exit 1
  HYPEROPT_AMD_LIB=${lib:-$PWD/hyperopt_amd/libtpe_hip.so} timeout -k 10 300 python -m pytest -q -x --timeout 120 tests/test_gpu_table.py tests/test_gpu_c5.py 2>&1 | tail -2 >> $out || exit 1
done
