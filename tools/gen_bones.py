"""Generate data/bones_90_16_v3.bin: buildFinal's 30 bone-cylinder endpoints for every frame
the reference's `./render final n` (n = 0..299 -> buildFinal(n*8)) and the default `./render`
(buildFinal(240)) use. Runs libdt's ASF/AMC forward kinematics (host_mocap.cpp, a
restatement of skeleton.cpp / motion.cpp / displaySkeleton.cpp) on the reference's mocap
files. Run in the build container only (/root/reference is absent on the GPU box).

Format: b"DTBONES <n_frames> <n_bones> <n_postures>\\n", int32[n_frames] posture ids,
then float64[n_frames][n_bones][6] (left xyz, right xyz).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("REF", "/root/reference")


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "distraytracer_amd", "libdt.so"))
    f = lib.dt_mocap_bone_table
    f.restype = ctypes.c_int
    asf = os.path.join(REF, "90.asf").encode()
    amc = os.path.join(REF, "90_16_v3.amc").encode()
    nb, npost = ctypes.c_int32(), ctypes.c_int32()
    rc = f(asf, amc, None, 0, None, ctypes.byref(nb), ctypes.byref(npost))
    if rc:
        sys.exit("mocap parse failed: %d" % rc)
    frames = sorted(set(min(n * 8, npost.value - 1) for n in range(300)))
    ids = np.array(frames, dtype=np.int32)
    out = np.zeros((len(frames), nb.value, 6), dtype=np.float64)
    rc = f(asf, amc, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(frames),
           out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(nb), ctypes.byref(npost))
    if rc:
        sys.exit("mocap FK failed: %d" % rc)
    path = os.path.join(ROOT, "data", "bones_90_16_v3.bin")
    with open(path, "wb") as fh:
        fh.write(b"DTBONES %d %d %d\n" % (len(frames), nb.value, npost.value))
        fh.write(ids.tobytes())
        fh.write(out.tobytes())
    print("wrote", path, len(frames), "frames x", nb.value, "bones; postures", npost.value)
    print("frame 240 bone 0:", out[frames.index(240), 0])


if __name__ == "__main__":
    main()
