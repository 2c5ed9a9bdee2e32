#!/bin/bash
# Round-4 GPU pass: parity suites, then the bench (only when the tests ended
# without a fault, abort or time limit: rc 0 or 1 = tests ran to the end).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r04}
SEL=${2:-tests/}
timeout -k 10 900 python -u -m pytest $SEL -q -m gpu --maxfail=15 --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -30 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
if [ "${3:-bench}" = "bench" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  brc=$?
  tail -c 3000 gpurun_out/${TAG}_bench.json; tail -5 gpurun_out/${TAG}_bench.err
  exit $brc
fi
exit $rc
