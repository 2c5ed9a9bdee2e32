cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in 65536 0; do
    TPE_LAT_PREFIX=$v timeout -k 10 200 python3 -u tools/rank_share.py 8 > gpurun_out/latprefix_${v}_${rep}.txt 2>&1 || exit 1
    echo "$v $rep $(grep -o 'projected_speedup_no_collective": [0-9.]*' gpurun_out/latprefix_${v}_${rep}.txt) $(grep '"N": 8, "max' gpurun_out/latprefix_${v}_${rep}.txt | grep -o '"max_rank_ms": [0-9.]*') $(grep '"N": 1, "max' gpurun_out/latprefix_${v}_${rep}.txt | grep -o '"max_rank_ms": [0-9.]*')"
  done
done
