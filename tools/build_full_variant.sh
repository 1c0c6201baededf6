#!/bin/bash
# build_full_variant.sh NAME [make variables...]: the whole product library from this tree's sources
# (every kernel instantiation), built in a scratch copy, as distraytracer_amd/variants/libdt_NAME.so,
# e.g. EXTRA="-DDT_X=1" for an A/B of a change that touches every instantiation.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
W=/tmp/fullvar_$name
rm -rf "$W"; mkdir -p "$W/distraytracer_amd" "$W/include"
cp -r "$R/distraytracer_amd/csrc" "$W/distraytracer_amd/"
rm -rf "$W/distraytracer_amd/csrc/build"
cp "$R"/include/*.h "$W/include/"
make -s -j8 -C "$W/distraytracer_amd/csrc" ../libdt.so "$@" 2>&1 | grep -v warning || true
mkdir -p "$R/distraytracer_amd/variants"
# copy then rename: a snapshot of the tree taken meanwhile (gpurun) never sees a half-written library
cp "$W/distraytracer_amd/libdt.so" "$R/distraytracer_amd/variants/.libdt_$name.so.tmp"
mv "$R/distraytracer_amd/variants/.libdt_$name.so.tmp" "$R/distraytracer_amd/variants/libdt_$name.so"
echo "built distraytracer_amd/variants/libdt_$name.so"
