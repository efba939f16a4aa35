R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
SKIP_BENCH=1 bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_tune.sh
