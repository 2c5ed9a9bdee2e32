cd $GRAFT_REPO_ROOT
out=gpurun_out/r02_variants.txt
: > $out
for f in "" tools/_variants/lib_*.so ""; do
  echo "== ${f:-base}" >> $out
  lib=${f:+$PWD/$f}
  TPE_SIDE_STREAM=0 HYPEROPT_AMD_LIB=${lib:-$PWD/hyperopt_amd/libtpe_hip.so} timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['group_ms'])" >> $out || exit 1
done
