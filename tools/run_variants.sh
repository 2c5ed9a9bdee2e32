#!/bin/bash
# GPU box: probe_table.py under every tools/_variants/lib_*.so (diagnostic).
#   tools/run_variants.sh <n_cand> <kinds>
cd "$(dirname "$0")/.."
for f in tools/_variants/lib_*.so; do
  echo "== $f"
  HYPEROPT_AMD_LIB=$PWD/$f timeout -k 10 120 python tools/probe_table.py $1 $2 table || exit 1
done
