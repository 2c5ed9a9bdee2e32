#!/bin/bash
# Kernel trace + separate PMC passes of one python command (GPU box, repo root).
#   tools/prof_pmc.sh <tag> <script.py> [args...]
# Each pass is its own rocprofv3 run under a hard limit; stops at the first failure.
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$tag
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 "$@" > $out/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $out/sq -o run -- python3 "$@" > $out/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $out/cache -o run -- python3 "$@" > $out/cache.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $out/fetch -o run -- python3 "$@" > $out/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run -- python3 "$@" > $out/write.log 2>&1
echo done
