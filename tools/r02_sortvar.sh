cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_posteriors.py tests/test_gpu_c5.py tests/test_gpu_history.py tests/test_gpu_parity.py > gpurun_out/t1.log 2>&1 || exit 1
for v in base SORT_NOMERGE; do
  if [ "$v" = base ]; then unset HYPEROPT_AMD_LIB; else export HYPEROPT_AMD_LIB=$PWD/tools/_variants/lib_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/sv_$v -o run -- python3 tools/rank_share.py --only 8 0 > gpurun_out/sv_$v.log 2>&1 || exit 1
done
unset HYPEROPT_AMD_LIB
timeout -k 10 100 python bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/n_1.json 2>/dev/null && timeout -k 10 200 python tools/rank_share.py 8 > gpurun_out/rs1.txt 2>&1
