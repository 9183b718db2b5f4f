#!/bin/bash
# One GPU-box session: build, parity tests, smoke, short bench, kernel profile.
# Every GPU step has its own time limit; steps are chained so the first
# failure ends the session.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -30 gpurun_out/build.log; exit 1; }
if [ "$STEP" = "all" ] || [ "$STEP" = "test" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -25 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -3 gpurun_out/bench.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "prof" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -20 {}'
fi
