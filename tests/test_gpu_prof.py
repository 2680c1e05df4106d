"""The library's profiling records (exacto_prof_read / exacto_prof_kernels, what bench.py's roofline block
reads): per family, the kernels that actually ran, named from their launch handles as rocprofv3 names
them, so the bench line's labels cannot drift from the library's launch choices (verdict r5 item 8)."""

import numpy as np
import pytest

from exacto_amd._ffi import HipContext
from bridge import uniform_residues

pytestmark = pytest.mark.gpu

Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]


def test_prof_kernels_name_what_ran(gpu_available):
    import torch
    n, B = 4096, 16
    rng = np.random.default_rng(5)
    ctx = HipContext(n, Q3, [], 65537, 1 << 16, device=0)
    rlk = uniform_residues(rng, (ctx.G, 2), Q3, n)
    ctx.load_relin_key(rlk)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()
    x, y = dev(uniform_residues(rng, (B, 2), Q3, n)), dev(uniform_residues(rng, (B, 2), Q3, n))
    out = torch.empty_like(x)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.bfv_mul_and_relin_dev(x, y, out, B)   # key conversion etc. outside the profiled call
    torch.cuda.synchronize()
    ctx.prof_enable(True)
    ctx.bfv_mul_and_relin_dev(x, y, out, B)
    torch.cuda.synchronize()
    recs = {k: ctx.prof_read(k) for k in (0, 1, 2, 4, 5, 6, 7, 8)}
    names = {k: ctx.prof_kernels(k) for k in recs}
    ctx.prof_enable(False)
    for k, r in recs.items():
        assert r["launches"] > 0, k
        got = names[k]
        assert got and sum(c for _, c, _ in got) == r["launches"], (k, got, r)
        assert all(nm.startswith("exacto::") and "(" not in nm for nm, _, _ in got), got
    fwd = [nm for nm, _, _ in names[0]]
    assert any(nm.startswith("exacto::ntt_fwd_pin_kernel<12") for nm in fwd), fwd
    assert names[2][0][0].startswith("exacto::ntt_inv_tensor"), names[2]
    assert names[8][0][0].startswith("exacto::ks32_crt_kernel<12, 3"), names[8]
    # a second read finds nothing new: the records were consumed
    assert ctx.prof_kernels(0) == []
