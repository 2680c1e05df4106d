"""The bench's exact production shapes against the C restatement (oracle/c), at the library's
DEFAULT chunking and pipeline lanes, called exactly as bench.py calls them (HipContext on the torch
stream, the key loaded from a device tensor, the `_dev` entry point over the whole batch).

The digests were written in the build container by `python tests/golden/make_golden.py
--bench-digests` (oracle/c: the exact BigInt schoolbook tensor for cfg3, eval.rs:113-147; the
literal HPS multiplier for compact_bfv / u64_dbfv, eval.rs:157-413; dbfv_mul with all d^2 products,
dbfv/eval.rs:82-149; the NTT product of ntt.rs:181-195 for cfg2).  The test regenerates the seeded
inputs, checks their digest, runs the GPU and compares the output digest; on a mismatch the per-block
digests name the rows that differ.

Which boundaries each batch crosses (context.hip chunk = products per pipeline chunk, scaled with
n (L + K); a batch that fits one chunk is split in halves over the two lanes):
  cfg3    B = 1024: two 512-product chunks, one per lane;
  cfg1    B = 8192: a 7168-product chunk and a 1024-product chunk, one per lane;
  u64dbfv B = 64 items = 4096 HPS products: four 1152-product chunks (18 items) and a 640-product one;
  cfg2    B = 16384 polys through ntt_polymul_kernel<12>;
  cfg4    B = 1024 dbfv_mul items (d = 2): 3072 products in six 512-product chunks over two lanes, the
          psum digit sums of an output limb spanning its item's products;
  cfg5    B = 8 depth-4 chains at n = 8192 (dbfv_mul_chain_dev, as bench.py calls it); each chain's
          output has its own digest (block = 1).
"""

import hashlib
import json
import os
import sys

import numpy as np
import pytest

from exacto_amd._ffi import HipContext

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
from make_golden import BENCH_DIGESTS, bench_digest_inputs, input_digest  # noqa: E402

# bench.py CONFIGS: (n, moduli, aux, plain, gadget base, dBFV (d, base, p))
Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]
BENCH = {
    "cfg1": (1024, [1099509805057], [562949953443841], 257, 1 << 16, None),
    "cfg2": (4096, [1152921504606830593], [], 65537, 1 << 16, None),
    "cfg3": (4096, Q3, [], 65537, 1 << 16, None),
    "u64dbfv": (4096, [1152921504606830593], [18014398509998081, 36028797018972161], 1040407, 256,
                (8, 256, 0)),
    "cfg4": (4096, Q3, [], 260111, 1 << 16, (2, 256, 65536)),
    "cfg5": (8192, Q3 + [1152921504606601217], [], 1040407, 256, (8, 256, 0)),
}


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


def _spec(name):
    with open(os.path.join(GOLD, "digests.json")) as f:
        return json.load(f)[name]


def _run(name, chunk=0):
    """The bench's call for BENCH_DIGESTS[name] on cuda:0; returns (spec, output as uint64)."""
    import torch
    spec = _spec(name)
    assert set(BENCH_DIGESTS[name]) <= set(spec), (name, "digests.json lacks keys of the spec")
    for k, v in BENCH_DIGESTS[name].items():
        assert spec[k] == v, (name, k)
    prm, x, y, rlk = bench_digest_inputs(spec)
    assert input_digest(x, y, rlk) == spec["sha256_inputs"]
    n, moduli, aux, plain, gbase, dbfv = BENCH[spec["config"]]
    B = spec["batch"]
    ctx = HipContext(n, moduli, aux, plain, gbase, device=0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    if chunk:
        ctx.set_chunk(chunk)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()
    dx, dy = dev(x), dev(y)
    out = torch.empty_like(dx)
    if rlk is not None:
        drlk = dev(rlk)
        torch.cuda.synchronize()
        ctx.load_relin_key_dev(drlk, rlk.shape[0])
    if spec["config"] == "cfg2":
        ctx.rns_polymul_dev(dx, dy, out, B)
    elif dbfv is None:
        ctx.bfv_mul_and_relin_dev(dx, dy, out, B)
    else:
        d, base, dplain = dbfv
        depth = spec.get("depth", 1)
        if depth == 1:
            ctx.dbfv_mul_dev(d, base, dplain, dx, dy, out, B)
        else:
            ctx.dbfv_mul_chain_dev(d, base, dplain, dx, dy, out, B, depth)
    ctx.synchronize()
    torch.cuda.synchronize()
    if dbfv is not None and spec["config"] in ("cfg4", "cfg5"):
        # the summed-digit key switch stays on, in the primary basis: cfg4's two-product
        # limbs in the narrow basis (bounded by the key's norms), cfg5's up-to-eight-product limbs in
        # the lazy one
        assert ctx.dbfv_key_switch == 1, ctx.dbfv_key_switch
    return spec, out.cpu().numpy().view(np.uint64)


def _check(spec, got):
    blk = spec["block"]
    bad = [i * blk for i, h in enumerate(spec["sha256_out_blocks"]) if sha(got[i * blk:(i + 1) * blk]) != h]
    assert not bad, f"{spec['config']}: row blocks of {blk} starting at {bad} differ from oracle/c"
    assert sha(got) == spec["sha256_out"]


@pytest.mark.parametrize("name", sorted(BENCH_DIGESTS))
def test_bench_shape_digest(gpu_available, name):
    spec, got = _run(name)
    _check(spec, got)


def test_u64_dbfv_chunk_invariance(gpu_available):
    """u64_dbfv at the bench's B = 64: one item per chunk (64 products), the default 1152, and one
    chunk holding the whole batch (4096) give the oracle's digest."""
    for chunk in (64, 1152, 4096):
        spec, got = _run("u64dbfv_bench", chunk=chunk)
        _check(spec, got)
