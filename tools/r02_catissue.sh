cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for m in pre post late; do
  echo "mode $m"
  TPE_CAT_ISSUE=$m timeout -k 10 100 python bench.py --no-extras --no-cpu-baseline --steps 60 2>/dev/null | tail -1 || exit 1
  TPE_CAT_ISSUE=$m timeout -k 10 100 python tools/rank_share.py --only 8 2 2>/dev/null | tail -1 || exit 1
done; done
