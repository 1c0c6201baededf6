#!/bin/bash
# Decodes the reference's JPEG textures with the reference's own vendored stb_image.h (v2.21,
# compiled unmodified into oracle/_ref/stb_decode by oracle/Makefile) so texel bytes match the
# reference's loadTexture (helpers.h:92-113). Output: data/textures/<file>.rgb (data fixture;
# /root/reference does not exist on the GPU box). Run in the build container only.
set -euo pipefail
cd "$(dirname "$0")/.."
REF=${REF:-/root/reference}
make -C oracle ref REF="$REF" >/dev/null
mkdir -p data/textures
for f in floor.jpeg sad_finder1_adj.jpg sad_finder2_adj.jpg; do   # the textures buildFinal loads
  oracle/_ref/stb_decode "$REF/textures/$f" "data/textures/$f.rgb"
done
