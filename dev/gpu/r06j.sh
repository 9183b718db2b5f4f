#!/bin/bash
# Round-6 A/B: firpfbch synthesizer M = 1024 with (base) and without (q0) the
# next block's X prefetched into registers during the transform; q0 also has
# the firpfbch2 synthesizer change of r06i (p0).  Parity of q0 after.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06j_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06j_ab.txt || exit 1; }
for i in 1 2; do
  for v in base q0; do
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfbsyn1 1024
    ab LQ_LIB_PATH=ab/$v/libliquid_mi355x.so AB_TAG=$v python dev/ab_r06.py pfbsyn 1024
  done
done
cat gpurun_out/r06j_ab.txt
LQ_LIB_PATH=ab/q0/libliquid_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "synthesizer or perfect_reconstruction" > gpurun_out/r06j_pytest.log 2>&1 || { tail -30 gpurun_out/r06j_pytest.log; exit 1; }
tail -2 gpurun_out/r06j_pytest.log
