#!/bin/bash
# Round-6 A/B: rows prefetched one group ahead in the firpfbch2 analyzers at
# M = 256 / 512 (8 rows per group: base 8, w1 6, w2 4) and M = 2048 (4 rows
# per group: base 4, w1 3, w2 2); parity of w1 / w2 after.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06n_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06n_ab.txt || exit 1; }
for i in 1 2; do
  for M in 256 512 2048; do
    for v in base w1 w2; do
      ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfb2 $M
    done
  done
done
cat gpurun_out/r06n_ab.txt
for v in w1 w2; do
  LQ_LIB_PATH=ab/$v/libliquid_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "firpfbch2_analyzer" > gpurun_out/r06n_pytest_$v.log 2>&1 || { tail -30 gpurun_out/r06n_pytest_$v.log; exit 1; }
  tail -2 gpurun_out/r06n_pytest_$v.log
done
