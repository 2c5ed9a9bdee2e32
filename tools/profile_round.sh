#!/bin/bash
# Kernel-trace summary + separate PMC passes for bench.py (run on the GPU box
# from the repo root).  Usage: tools/profile_round.sh <tag> [bench args...]
# Each pass is its own rocprofv3 run under a hard time limit; the script stops
# at the first failure.
set -e
tag=$1; shift
args=${*:---steps 3 --warmup 1 --no-cpu-baseline}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 bench.py $args > $out/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run -- python3 bench.py $args > $out/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run -- python3 bench.py $args > $out/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/sq -o run -- python3 bench.py $args > $out/sq.log 2>&1
# where the wave cycles go (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM -d $out/sq2 -o run -- python3 bench.py $args > $out/sq2.log 2>&1

# summarise on the box (the rocpd databases exceed what gpurun copies back)
python3 tools/rocpd_summary.py $out gpurun_out/${tag}
rm -rf $out/trace $out/fetch $out/write $out/sq $out/sq2
echo done
