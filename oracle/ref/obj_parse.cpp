// TEST INFRASTRUCTURE ONLY. Compiles the reference's vendored tiny_obj_loader.h, unmodified, from
// /root/reference (include path set by oracle/Makefile) into oracle/_ref/obj_parse, and parses an
// OBJ file through the ObjReader API exactly as the reference's loadObj does (objHelper.h:6-85:
// attrib.vertices / attrib.texcoords as tinyobj's real_t = float, three vertex and texcoord indices
// per face). Writes "DTOBJ <nv> <nt> <nf>\n" then nv*3 float, nt*2 float, nf*6 int32
// (v0 v1 v2 t0 t1 t2 per face). tests/test_oracle_obj.py compares the product loader's parse.
#define TINYOBJLOADER_IMPLEMENTATION
#include "tiny_obj_loader.h"
#include <cstdio>
#include <vector>

int main(int argc, char** argv)
{
  if (argc != 3) {
    fprintf(stderr, "usage: obj_parse in.obj out.bin\n");
    return 2;
  }
  tinyobj::ObjReaderConfig cfg;
  tinyobj::ObjReader reader;
  if (!reader.ParseFromFile(argv[1], cfg)) {
    fprintf(stderr, "TinyObjReader: %s\n", reader.Error().c_str());
    return 1;
  }
  const auto& attrib = reader.GetAttrib();
  const auto& shapes = reader.GetShapes();
  std::vector<int> faces;
  for (const auto& s : shapes) {
    size_t off = 0;
    for (size_t f = 0; f < s.mesh.num_face_vertices.size(); ++f) {
      const size_t fv = s.mesh.num_face_vertices[f];
      for (int k = 0; k < 3; ++k) faces.push_back(s.mesh.indices[off + k].vertex_index);
      for (int k = 0; k < 3; ++k) faces.push_back(s.mesh.indices[off + k].texcoord_index);
      off += fv;
    }
  }
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 1;
  const size_t nv = attrib.vertices.size() / 3, nt = attrib.texcoords.size() / 2, nf = faces.size() / 6;
  fprintf(o, "DTOBJ %zu %zu %zu\n", nv, nt, nf);
  fwrite(attrib.vertices.data(), sizeof(float), nv * 3, o);
  fwrite(attrib.texcoords.data(), sizeof(float), nt * 2, o);
  fwrite(faces.data(), sizeof(int), faces.size(), o);
  fclose(o);
  printf("%s: %zu vertices, %zu texcoords, %zu faces\n", argv[1], nv, nt, nf);
  return 0;
}
