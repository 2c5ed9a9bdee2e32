#!/bin/bash
# Interleaved bench A/B over variant trees (tools/mkvariant.sh): ms/step and
# the scorer's launch time from each tree's bench line.  Usage:
#   bash tools/ab_bench.sh . ab/x ab/y
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abb
for rep in 1 2; do
  for t in "$@"; do
    n=$( [ "$t" = "." ] && echo base || basename $t )
    ( cd $t && timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/abb/${n}_${rep}.json 2>/dev/null ) || exit 1
    echo "$n $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abb/${n}_${rep}.json) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/abb/${n}_${rep}.json) $(grep -o '"table_build": [0-9.]*' gpurun_out/abb/${n}_${rep}.json)"
  done
done
