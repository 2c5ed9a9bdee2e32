set -e
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r02b --steps 3 --warmup 1 --no-cpu-baseline --no-extras
echo ok
