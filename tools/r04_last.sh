#!/bin/bash
# Round-4 last pass on the final tree: GPU suite, the evidence of
# tools/r04_final.sh (bench, kernel-trace stats + PMC passes, rank share), C4.
cd $GRAFT_REPO_ROOT
TAG=${1:-r04_last}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --maxfail=10 --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/r04_final.sh $TAG || exit 1
timeout -k 10 400 python -u tools/scale_configs.py c4 > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || exit 1
tail -c 400 gpurun_out/${TAG}_c4.json
