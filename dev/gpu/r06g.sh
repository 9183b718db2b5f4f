#!/bin/bash
# Round-6 A/B: fused spgram kernel (spg0 = before, spg1 = register first-pass
# twiddles + in-register power partials, spg2 = the same with LDS twiddles),
# then the spgram parity tests on both variants.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06g_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06g_ab.txt || exit 1; }
for i in 1 2; do
  for v in spg0 spg1 spg2; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py spgram 1024
  done
done
cat gpurun_out/r06g_ab.txt
for v in spg1 spg2; do
  LQ_LIB_PATH=ab/$v/libliquid_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "spgram" > gpurun_out/r06g_pytest_$v.log 2>&1 || { tail -30 gpurun_out/r06g_pytest_$v.log; exit 1; }
  tail -2 gpurun_out/r06g_pytest_$v.log
done
