#!/bin/bash
# A/B of library variants on dev/ab/ab_pfb2m.py (dev tool): ab_pf.sh "M:m ..." dir1 dir2 ...
cd "$(dirname "$0")/../.."
ARGS=$1; shift
for rep in 1 2 3; do
  for d in "$@"; do
    echo -n "$d "; LQ_LIB_PATH=$d/libliquid_mi355x.so timeout -k 10 120 python dev/ab/ab_pfb2m.py $ARGS 2>&1 | grep -v amdgpu.ids | tail -1
  done
done
