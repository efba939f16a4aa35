#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel trace + PMC.
# Every GPU step has its own time limit; a crash/timeout ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 700 python -m pytest $TESTS -m gpu -q -rf -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
export TMPDIR=/tmp
P="$R/gpurun_out/prof"
rm -rf "$P"; mkdir -p "$P"
BARGS="--steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/kt" -o kt -- python3 "$R/bench.py" $BARGS > "$P/kt.log" 2>&1 || { echo ktrace failed; tail "$P/kt.log"; exit 5; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/fetch" -o fetch -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$P/fetch.log" 2>&1 || { echo pmc fetch failed; tail "$P/fetch.log"; exit 6; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/write" -o write -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$P/write.log" 2>&1 || { echo pmc write failed; tail "$P/write.log"; exit 7; }
find "$P" -name "*.csv" | head -20
echo done
