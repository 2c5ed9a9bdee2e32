# bench group times for the in-tree library and each tools/_variants/lib_*.so
cd $GRAFT_REPO_ROOT
out=gpurun_out/r02_variants.txt
echo "== base" > $out
timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['group_ms'])" >> $out || exit 1
for f in tools/_variants/lib_*.so; do
  echo "== $f" >> $out
  HYPEROPT_AMD_LIB=$PWD/$f timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['group_ms'])" >> $out || exit 1
done
echo "== base (again)" >> $out
timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['group_ms'])" >> $out || exit 1
