#!/bin/bash
# Round-6 A/B: matrix-core FIR with the prologue's loads drained before the
# chunk loop (f1), so the loop's waits leave the previous chunk's stores in
# flight (base: the loop header's merged wait counts drained them every
# chunk); then the firfilt parity tests on f1.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06o_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06o_ab.txt || exit 1; }
for i in 1 2; do
  for v in base f1; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py firfilt 64
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py firfilt 128
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py firfilt_rrrf 64
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py firfilt_cccf 64
  done
done
cat gpurun_out/r06o_ab.txt
LQ_LIB_PATH=ab/f1/libliquid_mi355x.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -k "firfilt or config1" > gpurun_out/r06o_pytest.log 2>&1 || { tail -30 gpurun_out/r06o_pytest.log; exit 1; }
tail -2 gpurun_out/r06o_pytest.log
