#!/bin/bash
# firfilt buffer-placement A/B over library variants (dev tool)
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for d in "$@"; do
    echo "== $d"; LQ_LIB_PATH=$d/libliquid_mi355x.so timeout -k 10 120 python dev/ab/ab_firalloc.py 2>&1 | grep -v amdgpu.ids
  done
done
