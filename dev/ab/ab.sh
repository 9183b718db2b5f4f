#!/bin/bash
# A/B timing of alternative library builds on one box (dev tool).  Each
# argument is a directory holding a libliquid_mi355x.so built from a variant
# (dev/ab/ab_build.sh); the bench runs alternate A B A B ... so box drift hits
# every variant alike.  Extra bench flags come from $AB_FLAGS.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
FLAGS=${AB_FLAGS:---no-extra --no-shard --no-percall --no-cpu-baseline}
for rep in 1 2; do
  for d in "$@"; do
    LQ_LIB_PATH=$d/libliquid_mi355x.so timeout -k 10 300 python bench.py $FLAGS > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
out = {'pfb2': d['roofline']['launch_ms']}
for k, v in d.items():
    if isinstance(v, dict) and 'roofline' in v:
        out[k] = v['roofline']['launch_ms']
    elif isinstance(v, dict) and 'launch_ms' in v:
        out[k] = v['launch_ms']
print('$d', {k: round(v, 4) for k, v in out.items()})"
  done
done
