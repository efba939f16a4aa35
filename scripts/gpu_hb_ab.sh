R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "heartbeat or Heartbeat or trace" -x -q --timeout 120 --timeout-method thread > gpurun_out/hb_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/hb_tests.log; exit 3; }
tail -2 gpurun_out/hb_tests.log
WL=heartbeat bash scripts/gpu_ab_libs.sh && WL=heartbeat bash scripts/gpu_ab_libs.sh > /dev/null
