# A/B of two builds of libtpe_hip.so on one box: ab/lib_old.so vs the in-tree
# library (table tests on the new one, then alternating bench lines and one
# kernel trace per build: average table-build / scorer durations).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_table.py tests/test_gpu_suggest.py tests/test_gpu_lattice.py -m gpu > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
NEW=$PWD/hyperopt_amd/libtpe_hip.so
OLD=$PWD/ab/lib_old.so
for v in old new old new; do
  if [ $v = old ]; then L=$OLD; else L=$NEW; fi
  HYPEROPT_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 40 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', round(d['ms_per_step'],4), round(d['suggest_p50_ms'],4))"
done
for v in old new; do
  if [ $v = old ]; then L=$OLD; else L=$NEW; fi
  HYPEROPT_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abprof_$v -o run -- python bench.py --no-cpu-baseline --no-extras --steps 20 > /dev/null 2>&1 || exit 1
  python - gpurun_out/abprof_$v <<'PY' || exit 1
import glob, re, sqlite3, sys
from collections import defaultdict
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
d = defaultdict(list)
for n, s, e in sqlite3.connect(db).execute("select name, start, end from kernels"):
    m = re.search(r"(k_\w+)", n)
    d[m.group(1) if m else n[:30]].append((e - s) / 1e3)
print(sys.argv[1], {k: round(sum(v) / len(v), 1) for k, v in d.items()
                    if k in ("k_table_build", "k_score_table_fast", "k_table_score", "k_score_slots")})
PY
done
