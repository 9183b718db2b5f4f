#!/bin/bash
# diagnostic: the firfilt [33-cccf] long-stream mismatch of r06o, f1 then base
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
for v in f1 base f1; do
  LQ_LIB_PATH=ab/$v/libliquid_mi355x.so timeout -k 10 120 python dev/dbg_fmx.py cccf 33 || exit 1
done
