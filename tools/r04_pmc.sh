#!/bin/bash
# Instruction counters of one kernel in one or more trees (one --pmc pass
# each, 8 SQ counters).  Usage: tools/r04_pmc.sh tag kernel_regex [tree ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; KRE=$2; shift 2
TREES=${*:-.}
ROOT=$PWD
for tree in $TREES; do
  name=$( [ "$tree" = "." ] && echo new || basename $tree )
  out=$ROOT/gpurun_out/$TAG/$name
  mkdir -p $out
  ( cd $tree && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH \
      --kernel-include-regex "$KRE" --output-format csv -d $out/pmc -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > $out/bench.json 2> $out/bench.err ) || exit $?
  ( cd $tree && PYTHONPATH=. timeout -k 10 120 python3 -u tools/r04_tstats.py > $out/tstats.log 2>&1 ) || exit $?
  echo "$name done"
done
