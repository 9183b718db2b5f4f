#!/bin/bash
# A/B of library variants on dev/ab/ab_msresamp.py (dev tool): ab_rs.sh dir1 dir2 ...
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for rep in 1 2 3; do
  for d in "$@"; do
    LQ_LIB_PATH=$d/libliquid_mi355x.so timeout -k 10 120 python dev/ab/ab_msresamp.py > gpurun_out/ab_rs.log 2>&1 || { tail -5 gpurun_out/ab_rs.log; exit 1; }
    python3 -c "
import json
out = {}
for l in open('gpurun_out/ab_rs.log'):
    if l.startswith('{'):
        d = json.loads(l); out[d['workload'].split('_crcf ')[0][:2] + d['workload'].split('r=')[1]] = d['ms']
print('$d', out)"
  done
done
