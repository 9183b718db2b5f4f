#!/bin/bash
# Round-6 A/B: firpfbch2 analyzer M = 1024 with the group's rows loaded at
# the top of its dot phase (a1) against one group ahead (base); firpfbch
# analyzer M = 1024 with the next group's rows issued after the dot phase's
# barrier (c1; c3: 8 of 16 rows) against before it (base, 12 of 16).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06k_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06k_ab.txt || exit 1; }
for i in 1 2; do
  for v in base a1; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfb2 1024
  done
  for v in base c1 c3; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfban1 1024
  done
done
cat gpurun_out/r06k_ab.txt
