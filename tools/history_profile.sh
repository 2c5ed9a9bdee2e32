#!/bin/bash
# Kernel trace + FETCH_SIZE / WRITE_SIZE passes of one tools/scale_configs.py
# config (c5: 100k-trial history; c4: 512 studies x 2k trials), summarised per
# kernel with the achieved HBM-side GB/s (tools/history_traffic.py).  Run on
# the GPU box from the repo root:  tools/history_profile.sh <tag> <config>
set -e
tag=$1; cfg=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/hist_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 tools/scale_configs.py $cfg > $out/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run -- python3 tools/scale_configs.py $cfg > $out/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run -- python3 tools/scale_configs.py $cfg > $out/write.log 2>&1
python3 tools/rocpd_summary.py $out gpurun_out/hist_${tag}
python3 tools/history_traffic.py gpurun_out/hist_${tag} > gpurun_out/hist_${tag}_traffic.txt
rm -rf $out/trace $out/fetch $out/write
cat gpurun_out/hist_${tag}_traffic.txt
