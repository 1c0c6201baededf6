/* TEST/DATA INFRASTRUCTURE ONLY. Compiles the reference's vendored stb_image.h (v2.21),
 * unmodified, from /root/reference (include path set by oracle/Makefile) into
 * oracle/_ref/stb_decode, which decodes the reference's JPEG textures exactly as the
 * reference's loadTexture (helpers.h:92-113) does. tools/gen_textures.sh writes the
 * decoded bytes to data/textures/*.rgb ("DTRGB <w> <h> <n>\n" + w*h*n bytes). */
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"
#include <stdio.h>

int main(int argc, char** argv)
{
  if (argc != 3) { fprintf(stderr, "usage: stb_decode in.jpg out.rgb\n"); return 2; }
  int w, h, n;
  unsigned char* d = stbi_load(argv[1], &w, &h, &n, 0);
  if (!d) { fprintf(stderr, "decode failed: %s\n", argv[1]); return 1; }
  FILE* f = fopen(argv[2], "wb");
  if (!f) { stbi_image_free(d); return 1; }
  fprintf(f, "DTRGB %d %d %d\n", w, h, n);
  fwrite(d, 1, (size_t)w * h * n, f);
  fclose(f);
  stbi_image_free(d);
  printf("%s: %dx%d n=%d\n", argv[1], w, h, n);
  return 0;
}
