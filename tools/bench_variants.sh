#!/bin/bash
# GPU box: bench.py group times under every tools/_variants/lib_*.so (diagnostic).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for f in hyperopt_amd/libtpe_hip.so tools/_variants/lib_*.so; do
  echo "== $f"
  HYPEROPT_AMD_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bv.json 2>/dev/null || echo FAILED
  python -c "import json; d=json.loads(open('gpurun_out/bv.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), d['group_ms'])"
done
