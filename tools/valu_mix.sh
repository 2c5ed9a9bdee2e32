#!/bin/bash
# Dynamic VALU instruction mix of bench.py's kernels by issue-cost class
# (PMC: the SQ_INSTS_VALU_* class counters, two passes of at most 8 SQ
# counters each, plus a kernel trace), summarised per kernel by
# tools/rocpd_summary.py.  Run on the GPU box from the repo root:
#     tools/valu_mix.sh <tag> [bench args...]
set -e
tag=$1; shift
args=${*:---steps 3 --warmup 1 --no-cpu-baseline --no-extras}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/mix_$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 bench.py $args > $out/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT -d $out/mixa -o run -- python3 bench.py $args > $out/mixa.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH -d $out/mixb -o run -- python3 bench.py $args > $out/mixb.log 2>&1
python3 tools/rocpd_summary.py $out gpurun_out/mix_${tag}
rm -rf $out/trace $out/mixa $out/mixb
echo done
