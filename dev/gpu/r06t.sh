#!/bin/bash
# Round-6 A/B: output stores of the M = 2048 / 4096 channelizer kernels with
# the non-temporal policy (base) or the default one (d0).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06t_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06t_ab.txt || exit 1; }
for i in 1 2; do
  for v in base d0; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfb2 2048
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfb2 4096
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfban1 4096
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfbsyn1 4096
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfbsyn 4096
  done
done
cat gpurun_out/r06t_ab.txt
