#!/bin/bash
# Round-end checks on one box (dev tool): the GPU suite, smoke(), the bench
# under the driver's command and at 50/20, the widened rows; each step under
# its own time limit, stopping at the first failure.  Writes gpurun_out/<tag>/.
cd "$(dirname "$0")/.."
TAG=${1:-final}
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_20_5.json 2> $OUT/bench_20_5.err || { tail -20 $OUT/bench_20_5.err; exit 1; }
timeout -k 10 600 python bench.py --steps 50 --warmup 20 --no-cpu-baseline > $OUT/bench_50_20.json 2> $OUT/bench_50_20.err || { tail -20 $OUT/bench_50_20.err; exit 1; }
timeout -k 10 400 python -u tools/bench_widened.py > $OUT/widened.txt 2> $OUT/widened.err || { tail -20 $OUT/widened.err; exit 1; }
echo done
