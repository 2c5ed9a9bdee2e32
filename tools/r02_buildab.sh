# A/B of two builds of libtpe_hip.so on one box: ab/lib_old.so vs the in-tree
# library (table tests on the new one, then alternating bench lines and one
# kernel-trace per build).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_table.py tests/test_gpu_suggest.py -m gpu > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
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
  HYPEROPT_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof_$v -o run -- python bench.py --no-cpu-baseline --no-extras --steps 20 > /dev/null 2>&1 || exit 1
  f=$(ls gpurun_out/abprof_$v/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/abprof_$v/run_kernel_stats.csv)
  echo "== $v"; grep -E "k_table_build|k_score_table_fast|k_lattice_sample|k_score_q" $f | cut -c1-160
done
