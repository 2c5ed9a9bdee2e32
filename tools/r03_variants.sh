#!/bin/bash
# A/B of diagnostic library builds (tools/diag_variants.sh) on the C3 bench:
# one line per variant with the table scorer's launch time and group times.
#   tools/r03_variants.sh <outdir> <variant>...   (variant: tools/_variants/lib_<v>.so, "base")
out=gpurun_out/$1; shift
mkdir -p $out
for v in "$@"; do
  lib=""
  [ "$v" != "base" ] && lib="HYPEROPT_AMD_LIB=$PWD/tools/_variants/lib_$v.so"
  env $lib timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extras > $out/$v.json 2> $out/$v.err || exit 1
  python -c "import json; d=json.loads(open('$out/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['group_ms'])" | tee -a $out/summary.txt
done
