#!/bin/bash
# A/B of HIP_FORCE_DEV_KERNARG (kernel arguments in device memory) on the
# bench step and the 8-way rank share, interleaved on one box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kab
for rep in 1 2; do
  for v in 1 0; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/kab/b_${v}_${rep}.json 2>/dev/null || exit 1
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python3 -u tools/rank_share.py 8 > gpurun_out/kab/rs_${v}_${rep}.txt 2>&1 || exit 1
    echo "kernarg=$v $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/kab/b_${v}_${rep}.json) $(grep -o 'projected_speedup_no_collective": [0-9.]*' gpurun_out/kab/rs_${v}_${rep}.txt) $(grep '"N": 8, "max' gpurun_out/kab/rs_${v}_${rep}.txt | grep -o '"max_rank_ms": [0-9.]*') $(grep '"N": 8, "max' gpurun_out/kab/rs_${v}_${rep}.txt | grep -o '"host_launch_ms": \[[0-9.]*')"
  done
done
