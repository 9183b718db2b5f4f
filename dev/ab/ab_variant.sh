#!/bin/bash
# Build a variant of the library that differs from the in-tree build only in
# the objects named (dev tool): ab_variant.sh <name> "<EXTRA flags>" obj1.o [obj2.o ...]
set -e
cd "$(dirname "$0")/../.."
name=$1; extra=$2; shift 2
mkdir -p ab/$name/obj
cp liquid-dsp_amd/obj/*.o ab/$name/obj/
for o in "$@"; do rm -f ab/$name/obj/$o; done
cd liquid-dsp_amd
make -s -j8 OBJ=../ab/$name/obj LIB=../ab/$name/libliquid_mi355x.so EXTRA="$extra"
