cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in post pre post pre; do
  echo "mode $m"
  TPE_CAT_ISSUE=$m HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python tools/scale_configs.py c4 2>/dev/null | tail -1 || exit 1
done
