#!/bin/bash
# Round-6 A/B: firpfbch2 M = 1024, seven rows prefetched (three pairs + one
# single row) and the eighth loaded in the dot phase (o1), against six + two
# (base); parity of o1 after.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06w_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06w_ab.txt || exit 1; }
for i in 1 2 3; do
  for v in base o1; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfb2 1024
  done
done
cat gpurun_out/r06w_ab.txt
LQ_LIB_PATH=ab/o1/libliquid_mi355x.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py -m gpu -q --timeout 120 --timeout-method thread -k "firpfbch2 or shard" > gpurun_out/r06w_pytest.log 2>&1 || { tail -30 gpurun_out/r06w_pytest.log; exit 1; }
tail -2 gpurun_out/r06w_pytest.log
