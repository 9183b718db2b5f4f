#!/bin/bash
# Round-6 A/B: the objects' history update folded into their stream kernels
# (main build) against its own launch after each call (base), per call with
# HIP events on the object's stream; then the full GPU suite on the main build.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06v_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06v_ab.txt || exit 1; }
for i in 1 2; do
  for v in base main; do
    L=ab/base/libliquid_mi355x.so; [ $v = main ] && L=liquid-dsp_amd/lib/libliquid_mi355x.so
    ab LQ_LIB_PATH=$L AB_TAG=$v python dev/ab_r06.py pfb2 1024
    ab LQ_LIB_PATH=$L AB_TAG=$v python dev/ab_r06.py firfilt 64
    ab LQ_LIB_PATH=$L AB_TAG=$v python dev/ab_r06.py resamp 1.037
    ab LQ_LIB_PATH=$L AB_TAG=$v python dev/ab_r06.py fftfilt 512
  done
done
cat gpurun_out/r06v_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06v_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06v_pytest.log
exit $rc
