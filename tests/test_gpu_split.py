"""GPU checks of the multi-GPU building blocks on one device:

* exacto_dbfv_mul_limbs (one GPU's output limbs of a split dbfv_mul, dbfv/eval.rs:109-132): every
  limb subset of a partition reproduces exacto_dbfv_mul's limbs bit for bit, at cfg4 and at cfg5's
  parameters (n = 1024), including the reduce folding of non-zero small representatives;
* the library's RCCL entry points with a one-rank communicator: unique id + comm init,
  exacto_ctx_broadcast_relin_key in place over the resident key, exacto_broadcast_galois_key and
  exacto_rccl_allgather_u64 (the multi-rank path is the driver's 8-GPU run; tests/test_dist.py
  covers the partition and the gather with gloo on CPU).
"""

import os

import numpy as np
import pytest

from exacto_amd._ffi import ExactoError, HipContext, RcclComm, rccl_unique_id
from exacto_amd.dist import limb_partition
from bridge import uniform_residues

pytestmark = pytest.mark.gpu

Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]
Q4 = Q3 + [1152921504606601217]


@pytest.mark.parametrize("n,q,plain,gbase,d,base,p,world", [
    (1024, Q3, 260111, 1 << 16, 2, 256, 65536, 2),        # cfg4 parameters, smaller ring
    (1024, Q4, 1040407, 256, 8, 256, 0, 3),               # cfg5 parameters, smaller ring
    (256, Q3, 1009, 1 << 16, 4, 7, 1000, 2),              # non-zero small representatives
])
def test_dbfv_mul_limbs_partition_matches_full(gpu_available, n, q, plain, gbase, d, base, p, world):
    rng = np.random.default_rng(31 + d)
    ctx = HipContext(n, q, [], plain, gbase)
    B = 3
    a = uniform_residues(rng, (B, d, 2), q, n)
    b = uniform_residues(rng, (B, d, 2), q, n)
    ctx.load_relin_key(uniform_residues(rng, (ctx.G, 2), q, n))
    full, _ = ctx.dbfv_mul(d, base, p, a, b)
    parts = limb_partition(d, world)
    assert sorted(k for ps in parts for k in ps) == list(range(d))
    for ls in parts:
        if not ls:
            continue
        got = ctx.dbfv_mul_limbs(d, base, p, a, b, ls)
        assert np.array_equal(got, full[:, ls]), ls
    # one limb at a time, and out-of-order lists
    assert np.array_equal(ctx.dbfv_mul_limbs(d, base, p, a, b, [d - 1, 0]), full[:, [d - 1, 0]])
    with pytest.raises(ExactoError):
        ctx.dbfv_mul_limbs(d, base, p, a, b, [d])
    with pytest.raises(ExactoError):
        ctx.dbfv_mul_limbs(d, base, p, a, b, [0, 0])


def test_rccl_one_rank_broadcast_and_allgather(gpu_available):
    import torch
    n = 1024
    rng = np.random.default_rng(9)
    src = HipContext(n, Q3, [], 65537, 0)
    dst = HipContext(n, Q3, [], 65537, 0)
    rlk = uniform_residues(rng, (src.G, 2), Q3, n)
    src.load_relin_key(rlk)
    ct1 = uniform_residues(rng, (2, 2), Q3, n)
    ct2 = uniform_residues(rng, (2, 2), Q3, n)
    want = src.bfv_mul_and_relin(ct1, ct2)
    comm = RcclComm(1, rccl_unique_id(), 0, 0)
    try:
        # with one rank the root's own resident key is the broadcast's source and destination: load it
        # on the device, broadcast in place (the key's auxiliary-basis forms are rebuilt after it)
        key = torch.from_numpy(rlk.view(np.int64)).cuda()
        torch.cuda.synchronize()
        dst.load_relin_key_dev(key, dst.G)
        dst.broadcast_relin_key(comm, 0, dst.G)
        dst.synchronize()
        assert np.array_equal(dst.bfv_mul_and_relin(ct1, ct2), want)
        # Galois key buffer broadcast in place and all-gather (one rank: recv = send)
        gk = torch.from_numpy(uniform_residues(rng, (3, 2), Q3, n).view(np.int64)).cuda()
        g0 = gk.clone()
        torch.cuda.synchronize()
        dst.broadcast_galois_key(comm, 0, gk, 3)
        send = torch.arange(1000, dtype=torch.int64, device="cuda")
        recv = torch.zeros(1000, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        dst.allgather_u64(comm, send, recv, 1000)
        dst.rccl_sync(comm)   # exacto_rccl_sync: the collective's completion under the deadline
        assert torch.equal(gk, g0) and torch.equal(recv, send)
        with pytest.raises(ExactoError):
            dst.broadcast_relin_key(comm, 1, dst.G)   # root out of range
        # a root whose resident key has another row count: the agreement step (every rank all-gathers
        # {num_keys, verdict} before any key is touched) rejects the call on every rank, key intact
        with pytest.raises(ExactoError) as e:
            dst.broadcast_relin_key(comm, 0, dst.G - 1)
        assert e.value.variant == "InvalidParam" and "rank 0 rejected" not in str(e.value)
        assert np.array_equal(dst.bfv_mul_and_relin(ct1, ct2), want)
        assert comm.count() == 1
    finally:
        comm.close()


_MISSING_RANK = r"""
import os, sys, time
sys.path.insert(0, os.environ["EXACTO_ROOT"])
from exacto_amd._ffi import ExactoError, RcclComm, rccl_unique_id
t0 = time.monotonic()
try:
    RcclComm(2, rccl_unique_id(), 0, 0)   # rank 1 never joins
    print("JOINED")
except ExactoError as e:
    print("ERR", round(time.monotonic() - t0, 1), str(e))
sys.stdout.flush()
os._exit(0)   # the init helper thread is still blocked in RCCL: no interpreter teardown
"""


def test_rccl_comm_init_deadline_when_a_rank_never_joins(gpu_available):
    """Verdict r5 item 6: a two-rank communicator whose second rank never joins fails with the library's
    deadline ($EXACTO_RCCL_TIMEOUT_S) instead of blocking forever (in a child process, which ends with
    os._exit: the abandoned init thread stays blocked in RCCL)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, EXACTO_RCCL_TIMEOUT_S="5", EXACTO_ROOT=root)
    r = subprocess.run([sys.executable, "-c", _MISSING_RANK], capture_output=True, text=True, timeout=90, env=env)
    out = r.stdout.strip().splitlines()
    assert out and out[-1].startswith("ERR"), (r.stdout[-1000:], r.stderr[-1000:])
    assert "timed out" in out[-1] and float(out[-1].split()[1]) < 30
