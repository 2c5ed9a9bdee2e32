cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "1 1" "1 2" "1 0" "1 2"; do set -- $v
TPE_CAT_EARLY=$1 TPE_NATIVE_LAUNCH=$2 HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python -c "
import sys, json; sys.path.insert(0, '.')
import bench
space = bench.c3_space(); vals, losses = bench.c3_history(space)
print('cat_early=$1 native=$2', json.dumps(bench.dropin_suggest_p50(space, vals, losses, bench.N_CAND, calls=30)))
" || exit 1
done
