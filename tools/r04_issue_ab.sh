#!/bin/bash
# A/B of the level's issue order knobs (TPE_CAT_ISSUE, TPE_CAT_EARLY) on the bench.
cd $GRAFT_REPO_ROOT
for v in "post 1" "late 1" "pre 1" "post 0"; do
  set -- $v
  r=$(TPE_CAT_ISSUE=$1 TPE_CAT_EARLY=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-extras --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')
  echo "issue=$1 early=$2 $r"
done
