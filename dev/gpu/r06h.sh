#!/bin/bash
# Round-6 A/B: firpfbch2 synthesizer M = 1024 (y0 = before; y8 / y12 / y16 =
# scaling folded into the transform's last pass, 8 / 12 / 16 of a block's 16
# values per lane prefetched during the column phase), then the synthesizer
# parity tests on y12 and y16.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06i_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06i_ab.txt || exit 1; }
for i in 1 2; do
  for v in base p0 p4 y8; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfbsyn 1024
  done
done
cat gpurun_out/r06i_ab.txt
for v in p0 p4; do
  LQ_LIB_PATH=ab/$v/libliquid_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "synthesizer or perfect_reconstruction" > gpurun_out/r06i_pytest_$v.log 2>&1 || { tail -30 gpurun_out/r06i_pytest_$v.log; exit 1; }
  tail -2 gpurun_out/r06i_pytest_$v.log
done
