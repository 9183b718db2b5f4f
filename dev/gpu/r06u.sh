#!/bin/bash
# Round-6 probe: firpfbch2 synthesizer M = 4096 with its X loads replaced by
# constants (nl; outputs wrong) against the shipped kernel: how much of the
# kernel's time the exposed X loads are.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06u_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06u_ab.txt || exit 1; }
for i in 1 2; do
  for v in base nl; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfbsyn 4096
  done
done
cat gpurun_out/r06u_ab.txt
