#!/bin/bash
# kernel-trace stats of a short bench run (profiles/<tag>_kernel_stats.csv)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
f=$(find gpurun_out/$TAG/prof -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/$TAG/kernel_stats.csv && head -25 gpurun_out/$TAG/kernel_stats.csv | cut -c1-160
exit $rc
