#!/bin/bash
# Per-variant VALU instruction counts of k_score_table_fast on the C3 bench
# (diagnostic libraries from tools/diag_variants.sh), one --pmc pass each,
# summarised on the box.   tools/r03_issue.sh <tag> <variant>...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/issue_$tag
mkdir -p $out
for v in "$@"; do
  lib=$PWD/hyperopt_amd/libtpe_hip.so
  [ "$v" != "base" ] && lib=$PWD/tools/_variants/lib_$v.so
  HYPEROPT_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $out/$v -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $out/$v.log 2>&1 || exit 1
  python3 - "$out/$v/run_results.db" "$v" >> $out/summary.txt <<'PY' || exit 1
import sqlite3, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
acc = defaultdict(list)
for name, cnt, val in c.execute("select kernel_name, counter_name, sum(value) from counters_collection "
                                "where kernel_name like '%k_score_table_fast%' group by dispatch_id, counter_name"):
    acc[cnt].append(val)
m = {k: sum(v) / len(v) for k, v in acc.items()}
cand = 30 * (1 << 22)
print(sys.argv[2], "valu/cand %.2f" % (m["SQ_INSTS_VALU"] * 64 / cand / 1.0 / 64 * 64 / 1),
      "waves %d" % m["SQ_WAVES"], "busy %.3f" % (m["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (m["GRBM_GUI_ACTIVE"] / 8)))
PY
  rm -rf $out/$v
done
cat $out/summary.txt
