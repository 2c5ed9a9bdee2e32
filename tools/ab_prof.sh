#!/bin/bash
# A/B kernel-trace stats over trees (default: the round-3 tree ab/r03 and this
# one), each with one stream (TPE_SIDE_STREAM=0: uncontended kernel times)
# and the default.  Usage: tools/ab_prof.sh tag [tree ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-ab}; shift
TREES=${*:-ab/r03 .}
ROOT=$PWD
for tree in $TREES; do
  name=$( [ "$tree" = "." ] && echo new || basename $tree )
  for side in ${SIDES:-0 1}; do
    out=$ROOT/gpurun_out/$TAG/${name}_s$side
    mkdir -p $out
    ( cd $tree && TPE_SIDE_STREAM=$side timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > $out/bench.json 2> $out/bench.err ) || exit $?
    echo "$name side=$side $(grep -o '"ms_per_step": [0-9.]*' $out/bench.json)"
  done
done
