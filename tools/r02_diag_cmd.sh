cd $GRAFT_REPO_ROOT
echo "== base" > gpurun_out/r02_diag.txt
timeout -k 10 120 python tools/probe_table.py 4194304 uniform,loguniform,normal table >> gpurun_out/r02_diag.txt 2>&1 || exit 1
for f in tools/_variants/lib_*.so; do
  echo "== $f" >> gpurun_out/r02_diag.txt
  HYPEROPT_AMD_LIB=$PWD/$f timeout -k 10 120 python tools/probe_table.py 4194304 uniform,loguniform,normal table >> gpurun_out/r02_diag.txt 2>&1 || exit 1
done
