#!/bin/bash
# r05: the two-pass qe_collect -- its parity tests, then the in-process timing
# of the main library against the three-pass variant (etcd_amd/lib/variants/).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05c2}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "collect" \
  --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/tests.log"; exit 2; }
tail -1 "$O/tests.log"
WL=ready_collect bash scripts/gpu_ab_libs.sh
