"""Generate tests/golden/noise_ref.npz from the REFERENCE's own noise.h (compiled unmodified by
oracle/Makefile into oracle/_ref/libref_noise.so). Inputs are seeded-random lattice points and
coordinates (negative ones included: truncation toward zero, int32 wrap in the hash) plus the
exact sample points of cloudColor's 200-step march for a few renderImageCloud rays. Run in the
build container (needs /root/reference); the fixture travels, the reference does not."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import oracle
    r = oracle.ref_noise()
    if r is None:
        sys.exit("oracle/_ref/libref_noise.so missing: make -C oracle ref")
    rng = np.random.default_rng(12345)
    n = 2000
    pi = rng.integers(0, 10, n).astype(np.int32)
    lat = rng.integers(-20000, 20000, (n, 3)).astype(np.int32)
    xyz = rng.uniform(-300, 300, (n, 3))
    xyz[:200] = rng.uniform(-2, 2, (200, 3))   # near the origin: sign changes of truncation
    noise = np.array([r.ref_Noise3D(int(i), *map(int, p)) for i, p in zip(pi, lat)])
    smooth = np.array([r.ref_Smoothed3D(int(i), *map(int, p)) for i, p in zip(pi, lat)])
    interp = np.array([r.ref_InterpolatedNoise3D(int(i), *map(float, p)) for i, p in zip(pi, xyz)])
    value = np.array([r.ref_ValueNoise_3D(*map(float, p)) for p in xyz])
    # cloudColor march points: p = 0 + z*ray, noise at (p.x, p.y, p.z + frame)
    zs = []
    z = np.float32(10.0)
    while z > 0:
        zs.append(z)
        z = np.float32(np.float64(z) - 0.05)
    rays = rng.uniform(-1.5, 1.5, (6, 3))
    rays[:, 2] = -1.0
    frames = np.array([1, 2, 7, 30, 240, 1952], dtype=np.float32)
    march_in = []
    for ray, fr in zip(rays, frames):
        for zz in zs:
            p = np.float64(zz) * ray
            march_in.append((p[0], p[1], p[2] + np.float64(fr)))
    march_in = np.array(march_in)
    march = np.array([r.ref_ValueNoise_3D(*map(float, p)) for p in march_in])
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "noise_ref.npz"), prime=pi, lattice=lat, xyz=xyz,
                        noise3d=noise, smoothed3d=smooth, interpolated3d=interp, value3d=value,
                        march_in=march_in, march_value=march, n_march_steps=len(zs))
    print("wrote", len(noise), "vectors +", len(march), "march points; steps per march:", len(zs))


if __name__ == "__main__":
    main()
