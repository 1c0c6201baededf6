"""Diagnostic: phase breakdown of the trace kernel from a -DDT_STAMPS build (DT_LIB=...)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distraytracer_amd as dt  # noqa: E402

NAMES = ["pop", "closest_hit", "hit+children", "occluded", "light loop rest", "sample (passes)", "sky",
         "-", "-", "-"]


def main():
    # config: c3 (default) or c4 (use_model, 256 spp)
    # optional: frame (buildFinal(frame), C5 frames: depth 10 as tools/animate.py) and WxH
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 240
    W, H = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1920x1080").split("x"))
    g = dt.globals_default()
    g.use_model = 1 if cfg == "c4" else 0
    b = dt.build_scene("final", frame, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = W, H, 256 if cfg == "c4" else 64, \
        8 if frame == 240 else 10, 2
    s = dt.Scene(b, g)
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = dt.render(s, g, frame, out)
    NS = 72 + 3 * 8 * 256
    arr = (ctypes.c_uint64 * NS)()
    dt.check(dt.lib.dt_debug_counters(s.handle, arr, NS))
    tot = arr[5] + arr[6]
    print("kernel ms %.2f" % st.kernel_ms)
    for i, n in enumerate(NAMES[:7]):
        print("%-18s %6.2f%%" % (n, 100.0 * arr[i] / max(tot, 1)))
    items = st.pixels * (4 if cfg == "c4" else 1)   # one wave item per 64 samples
    print("per wave item: DFS steps %.2f  wave-level prim tests %.2f  light iterations %.2f  node visits %.1f"
          % (arr[7] / items, arr[8] / items, arr[9] / items, st.wave_node_visits / items))
    names = {1: "sphere", 2: "cylinder", 3: "triangle", 4: "rectangle", 5: "prism", 6: "checker", 7: "checkerhole",
             0: "checkercyl"}
    print("closest-hit prim tests per item:", {names[t]: round(arr[10 + t] / items, 2) for t in range(8) if arr[10 + t]})
    print("shadow prim tests per item:", {names[t]: round(arr[18 + t] / items, 2) for t in range(8) if arr[18 + t]})
    print("shadow prim tests, lanes tested per item / hit fraction:",
          {names[t]: (round(arr[47 + t] / items, 1), round(arr[55 + t] / max(arr[47 + t], 1), 3)) for t in range(8) if arr[47 + t]})
    print("node visits per item: closest-hit %.1f  shadow %.1f" % (arr[26] / items, arr[27] / items))
    print("closest-hit root walks per item %.2f with %.1f node visits per walk; other walks %.1f visits per walk"
          % (arr[39] / items, arr[46] / max(arr[39], 1), (arr[26] - arr[46]) / max(arr[7] - arr[39], 1)))
    print("cycles in shadow leaf/prim blocks %.2f%%, closest-hit leaf/prim blocks %.2f%%"
          % (100.0 * arr[32] / max(tot, 1), 100.0 * arr[33] / max(tot, 1)))
    print("shadow grid per item: list tests %.1f, list walks %.2f, cell lookups inside %.2f / outside %.2f, "
          "list too long %.2f" % (arr[34] / items, arr[35] / items, arr[36] / items, arr[38] / items, arr[37] / items))
    print("scattered shadow waves per item %.2f, union walks %.2f; with a lane outside the grid %.2f (incl. "
          "coherent-check outside above)" % (arr[40] / items, arr[41] / items, arr[38] / items))
    print("wave-level shadow prim tests per item by path: cell list %.2f, union %.2f, tree walk %.2f, "
          "block subtree %.2f" % (arr[42] / items, arr[43] / items, arr[44] / items, arr[45] / items))
    print("block-subtree shadow walks per item %.2f (DT_SG_SUBTREE=1); gates per item: scattered waves with "
          "tree-walk lanes %.2f, subtrees built for the light %.2f, a lane outside the grid %.2f, a block without a "
          "subtree %.2f, more blocks than DT_SG_SUB_MULTI %.2f"
          % (arr[63] / items, arr[64] / items, arr[65] / items, arr[66] / items, arr[67] / items, arr[68] / items))
    print("shadow test cycles by path (%% of the kernel's): cell list %.2f%%, union %.2f%%, tree walks and other %.2f%%"
          % (100.0 * arr[69] / max(tot, 1), 100.0 * arr[70] / max(tot, 1), 100.0 * arr[71] / max(tot, 1)))
    print("shadow walks per item: all occluded %.2f (%.1f visits/walk), none occluded %.2f (%.1f/walk), total %.2f"
          % (arr[29] / items, arr[28] / max(arr[29], 1), arr[31] / items, arr[30] / max(arr[31], 1), arr[9] / items))
    # per (light, shape) shadow tests: wave-level tests per item, lanes per test, lane hit fraction
    d = b.desc
    rows = []
    for li in range(8):
        for sid in range(256):
            o = 72 + 3 * (li * 256 + sid)
            if arr[o]:
                rows.append((arr[o], li, sid, arr[o + 1], arr[o + 2]))
    rows = [r for r in rows if r[2] < 254]
    rows.sort(reverse=True)
    print("per light: calls/item, active lanes/call, occluded fraction, share of kernel cycles")
    for li in range(8):
        o = 72 + 3 * (li * 256 + 255)
        if arr[o]:
            sw = sum(r[0] for r in rows if r[1] == li)
            sl = sum(r[3] for r in rows if r[1] == li)
            print("  L%d %6.3f %5.1f %6.3f %6.2f%%   shape tests/item %.2f (%.1f lanes each)"
                  % (li, arr[o] / items, arr[o + 1] / arr[o], arr[o + 2] / max(arr[o + 1], 1),
                     100.0 * arr[o - 3] / max(tot, 1), sw / items, sl / max(sw, 1)))
    print("top shadow tests (light, shape, type): waves/item lanes/test hit-frac  v0 v2")
    for w, li, sid, ln, hi in rows[:30]:
        sh = d.shapes[sid] if sid < d.n_shapes else None
        ty = names.get(sh.type & 7, sh.type) if sh else "?"
        v0 = tuple(round(sh.v[0][k], 2) for k in range(3)) if sh else ()
        v2 = tuple(round(sh.v[2][k], 2) for k in range(3)) if sh else ()
        print("  L%d s%-3d %-11s %6.3f %5.1f %6.3f  %s %s" % (li, sid, ty, w / items, ln / w, hi / max(ln, 1), v0, v2))
    for li in range(d.n_lights):
        L = d.lights[li]
        print("  light %d type %d shape %d center %s A %s" % (li, L.type, L.shape_index,
              tuple(round(L.center[k], 2) for k in range(3)), tuple(round(L.A[k], 2) for k in range(3))))


if __name__ == "__main__":
    main()
