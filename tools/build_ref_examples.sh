#!/bin/bash
# Compile liquid-dsp's own example programs for the objects on this path,
# unchanged, against include/liquid.h (our drop-in header) and
# libliquid_mi355x.so -- the drop-in check.  Sources are read from
# /root/reference (this container only); binaries go to build/ref_examples/
# (git-ignored, shipped to the GPU box by gpurun), where
# tests/test_gpu_parity.py::test_reference_examples_run runs them.
set -euo pipefail
cd "$(dirname "$0")/.."
REF=${LIQUID_REFERENCE:-/root/reference}
[ -d "$REF/examples" ] || { echo "no reference examples at $REF: skipped"; exit 0; }
OUT=build/ref_examples
mkdir -p "$OUT"
LIBDIR=$PWD/liquid-dsp_amd/lib
EXAMPLES="dotprod_cccf dotprod_rrrf fftfilt_crcf firdecim_crcf firfilt_cccf firfilt_crcf firfilt_rrrf
          firinterp_crcf firpfbch2_crcf firpfbch_crcf firpfbch_crcf_analysis firpfbch_crcf_synthesis
          resamp_crcf resamp2_crcf resamp2_crcf_decim resamp2_crcf_filter resamp2_crcf_interp
          msresamp_crcf msresamp2_crcf fft firdes_kaiser firdespm nyquist_filter spgramcf spgramf"
for e in $EXAMPLES; do
  gcc -std=gnu99 -O2 -w -I include "$REF/examples/${e}_example.c" -L "$LIBDIR" -lliquid_mi355x \
      -Wl,-rpath,"$LIBDIR" -Wl,-rpath,'$ORIGIN/../../liquid-dsp_amd/lib' -lm -o "$OUT/${e}_example"
done
echo "built $(ls $OUT | wc -l) reference examples into $OUT"
