"""Per-kernel resource metadata of the built HIP code object (AMDGPU code-object notes):
VGPR/SGPR counts, VGPR/SGPR spills and the scratch (private segment) bytes per lane.

  python tools/kernel_resources.py [distraytracer_amd/csrc/build/dt_kernels.o] [--json out.json]

The object's .hip_fatbin section is unbundled for gfx950 (clang-offload-bundler) and its notes
read with llvm-readelf; no GPU needed."""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
        ".private_segment_fixed_size", ".group_segment_fixed_size")


def resources(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, hsaco = os.path.join(d, "fat.bin"), os.path.join(d, "k.hsaco")
        # objcopy rewrites its input when given no output file: dump from a scratch copy instead
        # (leaves the build's objects, and make's view of them, untouched)
        tmp_obj = os.path.join(d, "k.o")
        shutil.copyfile(obj, tmp_obj)
        subprocess.check_call(["objcopy", "--dump-section", ".hip_fatbin=" + fat, tmp_obj])
        subprocess.check_call([LLVM + "/clang-offload-bundler", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fat,
                               "--output=" + hsaco, "--unbundle"])
        notes = subprocess.check_output([LLVM + "/llvm-readelf", "--notes", hsaco]).decode()
    out, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*(\.[a-z_]+):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if line.lstrip().startswith("- "):
            cur = {}
        if k == ".name":
            out[v] = cur
        elif k in KEYS:
            cur[k[1:]] = int(v)
    return {k: v for k, v in out.items() if v}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    build = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distraytracer_amd", "csrc", "build")
    ap.add_argument("objects", nargs="*", default=[os.path.join(build, "dt_kernels.o"),
                                                   os.path.join(build, "dt_kernels_w5.o"),
                                                   os.path.join(build, "dt_kernels_rpc.o"),
                                                   os.path.join(build, "dt_kernels_dn.o"),
                                                   os.path.join(build, "dt_kernels_isect.o")])
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    r = {}
    for obj in a.objects:
        r.update(resources(obj))
    print(json.dumps(r, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(r, f, indent=1)
