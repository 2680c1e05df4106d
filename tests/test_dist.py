"""CPU multi-process test of the sharding / key-broadcast layer (gloo, world_size 2)."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from exacto_amd.dist import broadcast_key, gather_to, max_over_ranks, shard


def test_shard_covers_exactly():
    for total in (0, 1, 7, 1024, 1025):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = shard(total, r, world)
                seen.extend(range(s, s + c))
            assert seen == list(range(total))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # key made on rank 0 only, identical everywhere after the broadcast
        key = torch.arange(2 * 3 * 16, dtype=torch.int64).reshape(1, 2, 3, 16) if rank == 0 else \
            torch.zeros((1, 2, 3, 16), dtype=torch.int64)
        broadcast_key(key)
        ok_key = bool(torch.equal(key, torch.arange(96, dtype=torch.int64).reshape(1, 2, 3, 16)))
        # each rank "computes" its shard; the gather reassembles the global batch in order
        total = 5
        s, c = shard(total, rank, world)
        out = torch.arange(s, s + c, dtype=torch.int64).reshape(c, 1) * 10
        full = gather_to(out, total)
        ok_gather = True if rank != 0 else bool(torch.equal(full.flatten(), torch.arange(total) * 10))
        t = max_over_ranks(float(rank + 1))
        q.put((rank, ok_key, ok_gather, t))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_shard_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, ok_key, ok_gather, t in res:
        assert ok_key and ok_gather and t == 2.0


# ---------------------------------------------------------------- one dbfv_mul split by output limb

from exacto_amd.dist import gather_limbs, limb_partition, limb_products  # noqa: E402


def test_limb_partition_covers_and_balances():
    for d in (1, 2, 3, 8):
        for world in (1, 2, 3, 4, 8, 16):
            parts = limb_partition(d, world)
            assert len(parts) == world
            assert sorted(k for p in parts for k in p) == list(range(d))
            loads = [sum(limb_products(d)[k] for k in p) for p in parts]
            # LPT bound: no rank above the mean by more than the heaviest limb
            assert max(loads) <= sum(loads) / world + d
    assert limb_partition(8, 2) == [[0, 3, 4, 7], [1, 2, 5, 6]]   # 18 + 18 of cfg5's 36 products
    assert limb_partition(2, 2) == [[1], [0]]                     # cfg4: 2 products / 1 product


def _limb_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d, B = 5, 3
        parts = limb_partition(d, world)
        full = torch.arange(B * d * 4, dtype=torch.int64).reshape(B, d, 4)   # "limb k of item b"
        mine = parts[rank]
        compact = full[:, mine].clone()                                    # this rank's computed limbs
        out = gather_limbs(compact, parts, d)
        q.put((rank, bool(torch.equal(out, full))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_limbs(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_limb_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res)


# ---------------------------------------------------------------- bench.py's own launcher, sharding and timing

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env_extra=None):
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r


def test_bench_dry_gpus2_relaunches_torchrun():
    rc, line, r = _bench("--gpus", "2", "--dry", "--config", "cfg3", "--batch", "4", "--steps", "2", "--warmup", "1",
                         "--min-time", "0.1")
    assert rc == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["backend"] == "gloo"
    assert line["scaling"] == "weak" and line["config"]["global_batch"] == 8 and line["dry"] is True


def test_bench_dry_gpus2_limb_split_gathers_every_limb():
    rc, line, r = _bench("--gpus", "2", "--dry", "--config", "cfg5", "--split", "limbs", "--batch", "1",
                         "--steps", "2", "--warmup", "1", "--min-time", "0.1")
    assert rc == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["dry_gather_ok"] is True
    # one item: its limbs split 18 + 18 products over the two ranks, gathered after every chain step
    plan = line["config"]["split_plan"]
    assert plan["item_blocks"] == 1 and plan["limb_groups"] == 2
    assert plan["ranks"] == [[1, [0, 3, 4, 7]], [1, [1, 2, 5, 6]]]


def test_bench_dry_gpus8_cfg4_split_keeps_every_rank_busy():
    """Verdict r3 item 5: ONE cfg4 dbfv_mul batch (d = 2) over 8 ranks leaves no rank idle (items x
    limb groups), and every item's every limb is assembled on every rank (gloo, 8 CPU processes)."""
    rc, line, r = _bench("--gpus", "8", "--dry", "--config", "cfg4", "--split", "limbs", "--batch", "16",
                         "--steps", "2", "--warmup", "1", "--min-time", "0.1")
    assert rc == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 8 and line["dry_gather_ok"] is True
    ranks = line["config"]["split_plan"]["ranks"]
    assert len(ranks) == 8 and all(cnt > 0 and limbs for cnt, limbs in ranks)
    assert sum(cnt for cnt, _ in ranks) * 1 == 16 * line["config"]["split_plan"]["limb_groups"]


def test_split_plan_shapes():
    from exacto_amd.dist import split_plan
    # cfg4 batch over 8 ranks: whole items (no exchange between chain steps), 2 items each
    plan, pb, pl = split_plan(16, 2, 8)
    assert (pb, pl) == (8, 1) and all(c == 2 and ls == [0, 1] for _, c, ls in plan)
    # one cfg5 dbfv_mul on 8 ranks: one limb each, products 1..8 (the limb dimension is all there is)
    plan, pb, pl = split_plan(1, 8, 8)
    assert (pb, pl) == (1, 8) and sorted(k for _, _, ls in plan for k in ls) == list(range(8))
    # two cfg5 items on 4 ranks: 2 item blocks x 2 limb groups (18 products per rank), none idle
    plan, pb, pl = split_plan(2, 8, 4)
    assert (pb, pl) == (2, 2)
    assert all(c == 1 and sum(k + 1 for k in ls) == 18 for _, c, ls in plan)
    # a single cfg4 dbfv_mul cannot fill 8 ranks (3 products): least idle
    plan, pb, pl = split_plan(1, 2, 8)
    assert sum(1 for _, c, ls in plan if c and ls) == 2
    # every (item, limb) covered exactly once
    for B, d, world in ((5, 3, 6), (7, 8, 8), (3, 2, 4), (64, 8, 8)):
        plan, _, _ = split_plan(B, d, world)
        cover = sorted((b, k) for s0, c, ls in plan for b in range(s0, s0 + c) for k in ls)
        assert cover == [(b, k) for b in range(B) for k in range(d)]


def test_limb_products_follow_the_reps():
    """limb weights from the pair / coefficient rule of dbfv_plan: with nonzero small
    representatives the high pairs fold into low limbs (oracle/dbfv.py small_reps, reduce)."""
    from oracle import dbfv as odbfv
    for base, d, p in ((256, 2, 65536), (256, 8, 0), (7, 4, 1000), (3, 3, 20)):
        reps = odbfv.small_reps(base, d, p)
        want = [sum(1 for i in range(d) for j in range(d)
                    if i + j == k or (i + j >= d and reps[i + j - d][k] != 0)) for k in range(d)]
        assert limb_products(d, base, p) == want
    assert limb_products(8, 256, 0) == limb_products(8)   # zero reps: k + 1 pairs
    assert limb_products(4, 7, 1000) != limb_products(4)


def _plan_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from exacto_amd.dist import split_plan, gather_plan, torch_allgather
        B, d = 3, 5
        plan, _, _ = split_plan(B, d, world)
        full = torch.arange(B * d * 4, dtype=torch.int64).reshape(B, d, 4)
        s0, c, ls = plan[rank]
        compact = full[s0:s0 + c][:, ls].clone()
        out = torch.full_like(full, -1)
        gather_plan(compact, plan, rank, d, torch_allgather, out)
        q.put((rank, bool(torch.equal(out, full))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_gather_plan(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res)


def test_bench_world_size_mismatch_exits_nonzero():
    rc, line, _ = _bench("--gpus", "2", "--dry", env_extra={"WORLD_SIZE": "1"})
    assert rc != 0 and line is None


@pytest.mark.parametrize("phase", ["key_broadcast", "timed"])
def test_bench_dry_withheld_rank_exits_within_deadline(phase):
    """Verdict r5 item 6: one rank withholding its part of a collective (the key broadcast, or the
    barrier that opens the timed region) ends the job non-zero within about one deadline, with the
    watchdog's diagnostic line, instead of blocking it until the driver's time limit."""
    import time
    t0 = time.monotonic()
    rc, line, r = _bench("--gpus", "2", "--dry", "--config", "cfg3", "--batch", "4", "--steps", "2", "--warmup", "1",
                         "--min-time", "0.1",
                         env_extra={"EXACTO_BENCH_WITHHOLD": f"1:{phase}", "EXACTO_DIST_DEADLINE_S": "6"})
    dt = time.monotonic() - t0
    assert rc != 0 and line is None
    assert '"watchdog": "deadline exceeded"' in r.stderr and f'"phase": "{phase}"' in r.stderr, r.stderr[-2000:]
    assert dt < 150
