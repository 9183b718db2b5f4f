#!/bin/bash
# Compile liquid-dsp's own per-call benchmark bodies, unchanged, against
# include/liquid.h (our drop-in header) and libliquid_mi355x.so, and link
# them with tools/percall/percall_main.c into build/ref_bench/percall.
# Sources are read from /root/reference (this container only); the binary
# goes to build/ (git-ignored, shipped to the GPU box by gpurun), where
# bench.py's per_call leg runs it.  getrusage() is renamed so the driver's
# wall-clock hooks time exactly the reference's loops.
set -euo pipefail
cd "$(dirname "$0")/.."
REF=${LIQUID_REFERENCE:-/root/reference}
[ -d "$REF/src" ] || { echo "no reference sources at $REF: per-call harness skipped"; exit 0; }
OUT=build/ref_bench
mkdir -p "$OUT/obj"
LIBDIR=$PWD/liquid-dsp_amd/lib
SRCS="src/filter/bench/firfilt_crcf_benchmark.c src/filter/bench/firdecim_crcf_benchmark.c
      src/filter/bench/firinterp_crcf_benchmark.c src/filter/bench/resamp_crcf_benchmark.c
      src/filter/bench/resamp2_crcf_benchmark.c src/filter/bench/fftfilt_crcf_benchmark.c
      src/dotprod/bench/dotprod_rrrf_benchmark.c src/dotprod/bench/dotprod_crcf_benchmark.c
      src/dotprod/bench/dotprod_cccf_benchmark.c src/multichannel/bench/firpfbch_crcf_benchmark.c
      src/multichannel/bench/firpfbch2_crcf_benchmark.c src/buffer/bench/window_push_benchmark.c
      src/buffer/bench/window_read_benchmark.c"
DECLS=""; TABLE=""; OBJS=""
for s in $SRCS; do
  o="$OUT/obj/$(basename "$s" .c).o"
  gcc -std=gnu99 -O2 -w -I include -Dgetrusage=lqb_getrusage -c "$REF/$s" -o "$o"
  OBJS="$OBJS $o"
  for f in $(grep -oh "^void benchmark_[a-z0-9_]*" "$REF/$s" | sed 's/^void //' | sort -u); do
    DECLS="$DECLS void $f(struct rusage *, struct rusage *, unsigned long int *);"
    TABLE="$TABLE {\"${f#benchmark_}\", $f},"
  done
done
{ echo "#define LQB_DECLS $DECLS"; echo "#define LQB_TABLE $TABLE"; } > "$OUT/bench_table.h"
gcc -std=gnu99 -O2 -Wall -I "$OUT" tools/percall/percall_main.c $OBJS -L "$LIBDIR" -lliquid_mi355x \
    -Wl,-rpath,"$LIBDIR" -Wl,-rpath,'$ORIGIN/../../liquid-dsp_amd/lib' -lm -o "$OUT/percall"
echo "built $OUT/percall ($(echo "$TABLE" | grep -o '{' | wc -l) benchmarks)"
