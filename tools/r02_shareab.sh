# A/B of two library builds on the 8-way share (tools/rank_share.py 8) and
# N=1 bench, alternating on one box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NEW=$PWD/hyperopt_amd/libtpe_hip.so
OLD=$PWD/ab/lib_old.so
for v in old new old new old new; do
  if [ $v = old ]; then L=$OLD; else L=$NEW; fi
  HYPEROPT_AMD_LIB=$L HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python tools/rank_share.py 8 > gpurun_out/sab_$v.txt 2>/dev/null || exit 1
  echo "$v $(grep '"N": 8, "max_rank_ms"' gpurun_out/sab_$v.txt | cut -c1-48)"
done
for v in old new old new; do
  if [ $v = old ]; then L=$OLD; else L=$NEW; fi
  HYPEROPT_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 40 > gpurun_out/sab_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sab_$v.json'));print('$v N1', round(d['ms_per_step'],4), round(d['suggest_p50_ms'],4))"
done
