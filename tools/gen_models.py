"""Synthetic substitutes for the reference's missing ./models assets (the originals
live in a Dropbox folder and must not be fetched). buildFinal with use_model=true
(scene.h:258-602, finalBuildModels) loads:

  ./models/Column_LP_obj/Column_LP.obj                       -> two marble columns
  ./models/Column_LP_obj/Textures/Marble_Base_Color.jpg      -> their texture
  ./models/Column_LP_obj/Textures/Marble_Roughness.jpg       -> per-triangle roughness bytes
  ./models/helios_statue/helios_20.obj                       -> two busts on the columns

This script writes stand-ins of the same roles, deterministically, under data/models/:
  * a fluted column 1.3 units tall (the bust is placed at 3.9 = 3 * 1.3 above the floor,
    scene.h:471-474), with texture coordinates in [0, 1];
  * a bust (squashed icosphere head on a neck and a plinth), no texture coordinates;
  * marble base colour / roughness images in the repo's texture format (data/textures:
    "DTRGB w h n\\n" + bytes), the byte values stb_image would have produced.
Coordinates are written with 6 decimals, so every float parses to the same value with
strtof or tinyobj's parser. The reference renders with whatever the real assets contain;
these files only have to exercise the same code: OBJ ingest, per-vertex UV triangles,
textured Oren-Nayar shading, roughness from a map, and a few thousand BVH leaves.
"""
import math
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "data", "models")


def column_obj():
    """Fluted column: base plinth ring, shaft with 16 flutes, capital ring. Triangles only."""
    segs, rings = 32, 12
    height = 1.3
    verts, uvs, faces = [], [], []

    def radius(y, a):
        if y < 0.08 or y > height - 0.08:
            return 0.26                                # plinth / capital
        return 0.2 + 0.012 * math.cos(16 * a)          # flutes

    for r in range(rings + 1):
        y = height * r / rings
        for s in range(segs + 1):
            a = 2 * math.pi * s / segs
            rad = radius(y, a)
            verts.append((rad * math.cos(a), y, rad * math.sin(a)))
            uvs.append((s / segs, r / rings))
    row = segs + 1
    for r in range(rings):
        for s in range(segs):
            i0 = r * row + s
            i1, i2, i3 = i0 + 1, i0 + row, i0 + row + 1
            faces.append(((i0, i0), (i2, i2), (i1, i1)))
            faces.append(((i1, i1), (i2, i2), (i3, i3)))
    # caps (fan around a centre vertex, uv at the texture centre)
    for y, flip in ((0.0, True), (height, False)):
        c = len(verts)
        verts.append((0.0, y, 0.0))
        uvs.append((0.5, 0.5))
        base = 0 if y == 0.0 else rings * row
        for s in range(segs):
            a, b = base + s, base + s + 1
            faces.append(((c, c), (b, b), (a, a)) if flip else ((c, c), (a, a), (b, b)))
    return verts, uvs, faces


def bust_obj():
    """Icosphere head (2 subdivisions, squashed) on a cylinder neck and a box plinth."""
    t = (1 + 5 ** 0.5) / 2
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
         (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11),
         (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    v = [tuple(c / math.sqrt(sum(x * x for x in p)) for c in p) for p in v]
    for _ in range(2):
        cache, nf = {}, []

        def mid(a, b):
            k = (min(a, b), max(a, b))
            if k not in cache:
                p = [(v[a][i] + v[b][i]) / 2 for i in range(3)]
                n = math.sqrt(sum(x * x for x in p))
                v.append(tuple(x / n for x in p))
                cache[k] = len(v) - 1
            return cache[k]
        for a, b, c in f:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        f = nf
    head = [(0.16 * x, 0.55 + 0.2 * y, 0.18 * z) for x, y, z in v]
    faces = [tuple((i, None) for i in tri) for tri in f]
    verts = list(head)
    # neck: open cylinder from y=0.1 to y=0.42, r=0.07
    segs = 16
    n0 = len(verts)
    for y in (0.1, 0.42):
        for s in range(segs):
            a = 2 * math.pi * s / segs
            verts.append((0.07 * math.cos(a), y, 0.07 * math.sin(a)))
    for s in range(segs):
        a, b = n0 + s, n0 + (s + 1) % segs
        c, d = a + segs, b + segs
        faces.append(((a, None), (c, None), (b, None)))
        faces.append(((b, None), (c, None), (d, None)))
    # plinth box 0.36 x 0.1 x 0.3
    b0 = len(verts)
    for y in (0.0, 0.1):
        for x, z in ((-0.18, -0.15), (0.18, -0.15), (0.18, 0.15), (-0.18, 0.15)):
            verts.append((x, y, z))
    quads = [(0, 1, 2, 3), (4, 7, 6, 5), (0, 4, 5, 1), (1, 5, 6, 2), (2, 6, 7, 3), (3, 7, 4, 0)]
    for q in quads:
        a, b, c, d = (b0 + i for i in q)
        faces.append(((a, None), (b, None), (c, None)))
        faces.append(((a, None), (c, None), (d, None)))
    return verts, None, faces


def write_obj(path, verts, uvs, faces):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write("# synthetic stand-in (tools/gen_models.py)\n")
        for p in verts:
            fh.write("v %.6f %.6f %.6f\n" % p)
        if uvs:
            for t in uvs:
                fh.write("vt %.6f %.6f\n" % t)
        for tri in faces:
            if uvs:
                fh.write("f %s\n" % " ".join("%d/%d" % (vi + 1, ti + 1) for vi, ti in tri))
            else:
                fh.write("f %s\n" % " ".join("%d" % (vi + 1) for vi, _ in tri))


def marble(w, h, seed):
    """Veined marble: sin of a sum of octave sines (deterministic, no RNG)."""
    px = bytearray()
    for y in range(h):
        for x in range(w):
            u, v = x / w, y / h
            turb = sum(math.sin((u * 7.3 + v * 3.1) * (2 ** o) + seed * o) / (2 ** o) for o in range(5))
            vein = 0.5 + 0.5 * math.sin(12 * u + 5 * v + 3 * turb)
            g = int(200 + 50 * vein)
            px += bytes((min(255, g + 5), min(255, g), min(255, g - 8 if g > 8 else 0)))
    return px


def roughness(w, h):
    px = bytearray()
    for y in range(h):
        for x in range(w):
            g = int(90 + 80 * (0.5 + 0.5 * math.sin(x * 0.21) * math.cos(y * 0.17)))
            px += bytes((g, g, g))
    return px


def write_rgb(path, w, h, data):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as fh:
        fh.write(b"DTRGB %d %d 3\n" % (w, h))
        fh.write(bytes(data))


def main():
    col = os.path.join(OUT, "Column_LP_obj")
    write_obj(os.path.join(col, "Column_LP.obj"), *column_obj())
    write_rgb(os.path.join(col, "Textures", "Marble_Base_Color.jpg.rgb"), 128, 128, marble(128, 128, 0.7))
    write_rgb(os.path.join(col, "Textures", "Marble_Roughness.jpg.rgb"), 64, 64, roughness(64, 64))
    write_obj(os.path.join(OUT, "helios_statue", "helios_20.obj"), *bust_obj())
    print("wrote", OUT)


if __name__ == "__main__":
    main()
