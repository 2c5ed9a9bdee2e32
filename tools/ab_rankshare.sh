#!/bin/bash
# A/B over trees (default: ab/old and this one), interleaved, on one box: the
# 8-way rank share (tools/rank_share.py 8) and the bench line.
#   bash tools/ab_rankshare.sh [tree ...]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abrs
TREES=${*:-ab/old .}
for rep in 1 2; do
  for t in $TREES; do
    n=$( [ "$t" = "." ] && echo new || basename $t )
    ( cd $t && PYTHONPATH=. timeout -k 10 200 python3 -u tools/rank_share.py 8 > $GRAFT_REPO_ROOT/gpurun_out/abrs/${n}_${rep}_rs.txt 2>&1 ) || exit 1
    ( cd $t && timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/abrs/${n}_${rep}_bench.json 2>/dev/null ) || exit 1
    echo "$n $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abrs/${n}_${rep}_bench.json) $(grep -o '"band": [0-9.]*' gpurun_out/abrs/${n}_${rep}_bench.json) $(grep -o 'projected_speedup_no_collective": [0-9.]*' gpurun_out/abrs/${n}_${rep}_rs.txt) $(grep '"N": 8, "max' gpurun_out/abrs/${n}_${rep}_rs.txt | grep -o '"max_rank_ms": [0-9.]*') $(grep '"N": 1, "max' gpurun_out/abrs/${n}_${rep}_rs.txt | grep -o '"max_rank_ms": [0-9.]*')"
  done
done
