#!/bin/bash
# per-call legs of the reference's bench loops (default mode) + the
# small-call / firfilt parity tests
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 build/ref_bench/percall --runtime 0.25 firfilt_crcf_64 dotprod_crcf_64 dotprod_cccf_64 firpfbch2_crcf_a1024 firpfbch_crcf_a1024 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_small_calls.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "small or firfilt or example" > gpurun_out/r06pc_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06pc_pytest.log
exit $rc
