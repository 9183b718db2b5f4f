#!/bin/bash
# Round-6 A/B: rows prefetched one group ahead in the M = 1024 analyzers.
# firpfbch2 (8 rows per group): base 8, v1 4, v2 6 (the rest loaded in the
# dot phase).  firpfbch (16 rows per group, p = 8): base 12 issued before the
# barrier, v3 8 before, c3 8 after, v1 4 after, v2 6 after.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06l_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06l_ab.txt || exit 1; }
for i in 1 2; do
  for v in base v1 v2; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfb2 1024
  done
  for v in base v3 c3 v1 v2; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfban1 1024
  done
done
cat gpurun_out/r06l_ab.txt
