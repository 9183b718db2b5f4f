#!/bin/bash
# Round-6: firpfbch2 per-call (one block per call) on the signalled
# one-launch path; then the firpfbch2 / examples / small-call tests.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 build/ref_bench/percall --runtime 0.25 firpfbch2_crcf_a1024 firpfbch_crcf_a1024 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_small_calls.py tests/test_gpu_shard.py -m gpu -q --timeout 120 --timeout-method thread -k "firpfbch or example or shard or small" > gpurun_out/r06y_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06y_pytest.log
exit $rc
