#!/bin/bash
# Round-6 GPU session: parity suite (optionally a subset), smoke, bench under
# the driver's command.  Every GPU step has its own time limit and the first
# failure ends the session.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06}
SEL=${2:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
cat gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench.log
