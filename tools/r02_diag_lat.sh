cd $GRAFT_REPO_ROOT
echo "== base" > gpurun_out/r02_diag_lat.txt
timeout -k 10 120 python tools/probe_lattice_diag.py >> gpurun_out/r02_diag_lat.txt 2>&1 || exit 1
for f in tools/_variants/lib_*.so; do
  echo "== $f" >> gpurun_out/r02_diag_lat.txt
  HYPEROPT_AMD_LIB=$PWD/$f timeout -k 10 120 python tools/probe_lattice_diag.py >> gpurun_out/r02_diag_lat.txt 2>&1 || exit 1
done
