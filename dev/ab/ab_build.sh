#!/bin/bash
# Build the library from the working tree into ab/<name>/ (dev tool; see dev/ab/ab.sh).
set -e
cd "$(dirname "$0")/../../liquid-dsp_amd"
make -s -j8 OBJ=../ab/$1/obj LIB=../ab/$1/libliquid_mi355x.so EXTRA="$2"
