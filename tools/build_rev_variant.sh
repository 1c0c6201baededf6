#!/bin/bash
# build_rev_variant.sh NAME [REV]: the whole product library of git revision REV (default HEAD) built
# in a scratch worktree, as distraytracer_amd/variants/libdt_NAME.so: the same-box A/B baseline
# (DT_LIB=...) for the working tree's changes.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:-HEAD}
W=/tmp/revvar_$name
git -C "$R" worktree remove --force "$W" 2>/dev/null || rm -rf "$W"
git -C "$R" worktree add --detach "$W" "$rev" >/dev/null
make -s -j8 -C "$W/distraytracer_amd/csrc" ../libdt.so 2>&1 | grep -v warning || true
mkdir -p "$R/distraytracer_amd/variants"
cp "$W/distraytracer_amd/libdt.so" "$R/distraytracer_amd/variants/.libdt_$name.so.tmp"
mv "$R/distraytracer_amd/variants/.libdt_$name.so.tmp" "$R/distraytracer_amd/variants/libdt_$name.so"
git -C "$R" worktree remove --force "$W"
echo "built distraytracer_amd/variants/libdt_$name.so from $(git -C "$R" rev-parse --short "$rev")"
