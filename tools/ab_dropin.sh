#!/bin/bash
# Interleaved A/B of the drop-in figures (bench.py's dropin_suggest and
# append_step) over trees: bash tools/ab_dropin.sh ab/old .
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abd
for rep in 1 2; do
  for t in "$@"; do
    n=$( [ "$t" = "." ] && echo new || basename $t )
    ( cd $t && timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/abd/${n}_${rep}.json 2>/dev/null ) || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/abd/${n}_${rep}.json').read().strip().splitlines()[-1]); print('$n $rep', round(d['ms_per_step'],4), 'dropin', round(d['dropin_suggest']['p50_ms'],4), 'append', round(d['append_step']['p50_ms'],4), 'readme', round(d['readme_suggest']['p50_ms'],4))"
  done
done
