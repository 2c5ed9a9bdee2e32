#!/bin/bash
# Quick A/B of bench.py group timings (GPU box, repo root): one line per run
#   tools/quick_groups.sh <outdir> <VAR=value>...   (each arg: env for one run)
out=gpurun_out/$1; shift
mkdir -p $out
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline > $out/b$i.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$out/b$i.log').read().strip().splitlines()[-1]); print('$envs', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['group_ms'], round(d['dropin_suggest']['p50_ms'],3))"
done
