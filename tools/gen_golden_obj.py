"""Generate tests/golden/obj_tinyobj.npz: the substitute OBJ models (data/models, tools/gen_models.py)
parsed by the REFERENCE's own vendored tiny_obj_loader.h (compiled unmodified by oracle/Makefile into
oracle/_ref/obj_parse, used through the ObjReader API as objHelper.h:6-85 uses it). Run in the build
container (needs /root/reference); the fixture travels, the reference does not."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODELS = ["Column_LP_obj/Column_LP.obj", "helios_statue/helios_20.obj"]


def tinyobj_parse(path):
    """(vertices float32[n,3], texcoords float32[n,2], faces int32[n,6]) from oracle/_ref/obj_parse"""
    exe = os.path.join(ROOT, "oracle", "_ref", "obj_parse")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "o.bin")
        subprocess.check_call([exe, path, out], stdout=subprocess.DEVNULL)
        raw = open(out, "rb").read()
    head, body = raw.split(b"\n", 1)
    nv, nt, nf = map(int, head.split()[1:])
    v = np.frombuffer(body, np.float32, nv * 3, 0).reshape(nv, 3)
    t = np.frombuffer(body, np.float32, nt * 2, nv * 12).reshape(nt, 2)
    f = np.frombuffer(body, np.int32, nf * 6, nv * 12 + nt * 8).reshape(nf, 6)
    return v, t, f


def main():
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "obj_parse")):
        sys.exit("oracle/_ref/obj_parse missing: make -C oracle ref")
    arrays = {}
    for i, m in enumerate(MODELS):
        v, t, f = tinyobj_parse(os.path.join(ROOT, "data", "models", m))
        arrays["v%d" % i], arrays["t%d" % i], arrays["f%d" % i] = v, t, f
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "obj_tinyobj.npz"), models=np.array(MODELS), **arrays)
    print("wrote tests/golden/obj_tinyobj.npz")


if __name__ == "__main__":
    main()
