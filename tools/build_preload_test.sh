#!/bin/bash
# LD_PRELOAD check (tests/test_gpu_preload.py): a stand-in libliquid.so and a
# program linked against it; the test runs the program with and without
# LD_PRELOAD=libliquid_mi355x.so.  Outputs go to build/preload/ (git-ignored).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=build/preload
mkdir -p "$OUT"
gcc -std=gnu99 -O2 -fPIC -shared tests/preload/liquid_stub.c -o "$OUT/libliquid.so"
gcc -std=gnu99 -O2 -w -I include tests/preload/prog.c -L "$OUT" -lliquid -Wl,-rpath,'$ORIGIN' -lm -o "$OUT/prog"
echo "built $OUT/prog against the stand-in $OUT/libliquid.so"
