#!/bin/bash
# Round-6 A/B: matrix-core FIR, the next chunk's loads issued after this
# chunk's four tile stores (p1) instead of before its MFMAs (base).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06s_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06s_ab.txt || exit 1; }
for i in 1 2; do
  for v in base p1; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py firfilt 64
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py firfilt_cccf 64
  done
done
cat gpurun_out/r06s_ab.txt
