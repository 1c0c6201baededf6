"""C5 animation frames at their own settings but a small image (tools/parity_sweep.py runs all 300):
buildFinal(n*8) for n across the room, the room-to-tunnel transition (deep glossy cascades, also
through the work-sharing kernel), the tunnel with linear and cubic motion blur and the cloud frames
(the builder's 1 spp), 64 spp and depth 10 elsewhere, each with the build dt_render selects (the
called sky march of the tunnel builds among them) against the oracle, bit for bit, same ray count."""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle
from parity_check import assert_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 60, 121, 136, 150, 180, 210, 240, 260])
def test_animation_frame(cuda, n):
    g = dt.globals_default()
    g.use_model = 0
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 64, 36, 64, 10
    built = dt.build_scene("final", n * 8, g)
    s = dt.Scene(built, g)
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = dt.render(s, g, n * 8, out)
    gpu = out.cpu().numpy()
    dn = None
    if 121 <= n <= 139:
        s.set_kernel(dt.DT_KERNEL_DONATE)
        out.zero_()
        st_dn = dt.render(s, g, n * 8, out)
        dn = out.cpu().numpy()
    name = dt.trace_build(built, g, n * 8)[0]
    s.close()
    ref, rst = oracle.render(built, g, n * 8, dt.tiles())
    assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
    assert_parity("C5 frame %d (%s, %d spp)" % (n * 8, name, g.antialias_samples), gpu, ref)
    if dn is not None:
        assert st_dn.rays == rst.rays
        assert_parity("C5 frame %d (work-sharing kernel)" % (n * 8), dn, ref)
