#!/bin/bash
# A/B: rank share (8-way) and bench on the old tree vs this one, interleaved
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abrs
for rep in 1 2; do
  for t in ab/old .; do
    n=$( [ "$t" = "." ] && echo new || echo old )
    ( cd $t && PYTHONPATH=. timeout -k 10 200 python3 -u tools/rank_share.py 8 > $GRAFT_REPO_ROOT/gpurun_out/abrs/${n}_${rep}_rs.txt 2>&1 ) || exit 1
    ( cd $t && timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/abrs/${n}_${rep}_bench.json 2>/dev/null ) || exit 1
    echo "$n $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abrs/${n}_${rep}_bench.json) $(grep -o 'projected_speedup_no_collective": [0-9.]*' gpurun_out/abrs/${n}_${rep}_rs.txt) $(grep '"N": 8, "max' gpurun_out/abrs/${n}_${rep}_rs.txt | grep -o '"max_rank_ms": [0-9.]*') $(grep '"N": 1, "max' gpurun_out/abrs/${n}_${rep}_rs.txt | grep -o '"max_rank_ms": [0-9.]*')"
  done
done
