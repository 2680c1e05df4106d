"""Multi-GPU layer: one process per GPU, batches sharded across ranks, keys broadcast.

The path shards embarrassingly (every bfv_mul_and_relin / dbfv_mul in a batch is
independent), so batch sharding has NO data-path collective: each rank owns a
contiguous slice of the batch.  The only collective there is the one-time broadcast of the
relinearisation key over xGMI (2.25 MiB at cfg3/4, 15 MiB at cfg5), made by the library itself
(``HipContext.broadcast_relin_key``: ncclBroadcast into the resident key) or by torch.distributed.

One dbfv_mul can also be split across GPUs (north_star: "the d^2 digit-pair muls of a single
dbfv_mul shard across the GPUs"): output limb k = sum over pairs (i, j) with i + j = k
(dbfv/eval.rs:109-132), so assigning whole output limbs to ranks needs no cross-GPU sum
(``limb_partition``); each rank computes its limbs (``HipContext.dbfv_mul_limbs_dev``) and
``gather_limbs`` all-gathers them (never an RCCL sum, which would overflow mod q).
"""

from __future__ import annotations

import json
import os
import sys
import threading
import time

import torch
import torch.distributed as dist


def deadline_s() -> float:
    """Deadline of one phase of the multi-rank path, seconds ($EXACTO_DIST_DEADLINE_S, default 600)."""
    return float(os.environ.get("EXACTO_DIST_DEADLINE_S", "600"))


class Watchdog:
    """Deadline per phase of a multi-rank run.

    A daemon thread checks the armed phase twice a second.  When a phase outlives its deadline (a
    rank never joined a collective, a communicator init or an RCCL kernel is stuck) it prints one JSON
    diagnostic line to stderr and ends the process with ``os._exit(124)``: no exec, no interpreter
    teardown that could block again in the same collective.  torchrun then sees a failed rank and stops
    the others, so the whole job exits non-zero within about one deadline.  Native calls release the
    GIL (ctypes, torch.distributed), so the thread runs while the main thread is blocked in them.

    Test hook (``--dry`` runs only): ``EXACTO_BENCH_WITHHOLD=<rank>:<phase>`` makes that rank stall at the
    start of that phase, i.e. withhold its part of the phase's collective."""

    def __init__(self, rank: int, enabled: bool = True, withhold_ok: bool = False):
        self.rank = rank
        self.phase = None
        self.deadline = None
        self.t0 = None
        self._lock = threading.Lock()
        w = os.environ.get("EXACTO_BENCH_WITHHOLD", "") if withhold_ok else ""
        self._withhold = tuple(w.split(":", 1)) if ":" in w else None
        if enabled:
            threading.Thread(target=self._run, name="exacto-watchdog", daemon=True).start()

    def arm(self, phase: str, seconds: float | None = None):
        with self._lock:
            self.phase, self.t0 = phase, time.monotonic()
            self.deadline = self.t0 + (deadline_s() if seconds is None else seconds)
        if self._withhold and self._withhold == (str(self.rank), phase):
            while True:   # withholding this rank's part: only the watchdog ends this
                time.sleep(3600)

    def disarm(self):
        with self._lock:
            self.phase = self.deadline = None

    def _run(self):
        while True:
            time.sleep(0.5)
            with self._lock:
                ph, dl, t0 = self.phase, self.deadline, self.t0
            if dl is not None and time.monotonic() > dl:
                sys.stderr.write(json.dumps({"watchdog": "deadline exceeded", "rank": self.rank, "phase": ph,
                                             "waited_s": round(time.monotonic() - t0, 1)}) + "\n")
                sys.stderr.flush()
                sys.stdout.flush()
                os._exit(124)


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, start+count) slice of ``total`` items for ``rank`` (sizes differ by <= 1)."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def broadcast_key(key: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Broadcast the relinearisation key (``[G][2][L][n]`` int64 view of u64) from ``src``."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(key, src=src)
    return key


def load_key_everywhere(ctx, key: torch.Tensor, num_keys: int, src: int = 0):
    """Broadcast ``key`` from ``src`` and make it the context's resident relinearisation key."""
    broadcast_key(key, src)
    ctx.load_relin_key_dev(key, num_keys)


def rccl_comm_for(ctx, device: int):
    """An RCCL communicator of the library (exacto_rccl_comm_init) over the torch.distributed
    group: rank 0's unique id is broadcast over the default group, every rank joins on ``device``."""
    from exacto_amd._ffi import RcclComm, rccl_unique_id
    world, rank = dist.get_world_size(), dist.get_rank()
    uid = rccl_unique_id() if rank == 0 else bytes(128)
    be = dist.get_backend()
    t = torch.tensor(list(uid), dtype=torch.uint8, device=torch.device("cuda", device) if be == "nccl" else "cpu")
    dist.broadcast(t, src=0)
    return RcclComm(world, bytes(t.cpu().tolist()), rank, device)


def max_over_ranks(value: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to(shard_out: torch.Tensor, total: int, dst: int = 0):
    """Collect every rank's output shard on ``dst`` only (returns the concatenation there, None
    elsewhere): a gather, so no other rank holds the whole batch.  Shards are padded to the largest
    shard size for the collective."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    maxc = shard(total, 0, world)[1]
    pad = torch.zeros((maxc,) + tuple(shard_out.shape[1:]), dtype=shard_out.dtype, device=shard_out.device)
    pad[: shard_out.shape[0]] = shard_out
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, parts, dst=dst)
    if rank != dst:
        return None
    return torch.cat([parts[r][: shard(total, r, world)[1]] for r in range(world)])


def small_reps(base: int, d: int, plain: int) -> list[list[int]]:
    """reps[j - d] = the base-b digits of base^j mod p for j = d .. 2d-2 (lattice.rs:104-122
    compute_simple; p = 0 is 2^64 by wrapping_pow), as exacto_hip's dbfv_plan computes them."""
    reps = []
    for j in range(d, 2 * d - 1):
        val = pow(base, j, 1 << 64) if plain == 0 else pow(base, j, plain)
        dg = []
        for _ in range(d):
            dg.append(val % base)
            val //= base
        reps.append(dg)
    return reps


def limb_products(d: int, base: int | None = None, plain: int | None = None) -> list[int]:
    """Products each output limb k < d of a dbfv_mul needs: the pairs (i, j) with a nonzero
    coefficient for k -- 1 when i + j = k, reps[i + j - d][k] when i + j >= d (the reduce folding,
    reduction.rs:34-52) -- the same rule as the library's dbfv_plan.  Without (base, plain) the
    small representatives are taken as all zero (every BASELINE dBFV config): k + 1 pairs."""
    reps = small_reps(base, d, plain) if base is not None else None
    out = []
    for k in range(d):
        cnt = 0
        for i in range(d):
            for j in range(d):
                s = i + j
                coef = 1 if s == k else (reps[s - d][k] if (reps is not None and s >= d) else 0)
                cnt += coef != 0
        out.append(cnt)
    return out


def limb_partition(d: int, world: int, weights=None) -> list[list[int]]:
    """Output limbs of one dbfv_mul per rank, balanced by product count (longest-processing-time
    greedy: heaviest limb first onto the least-loaded rank, ties to the lower rank).  Every limb
    goes to exactly one rank; ranks beyond d limbs get none.  Deterministic, so every rank
    computes the same partition without communicating."""
    w = limb_products(d) if weights is None else list(weights)
    load = [0] * world
    parts: list[list[int]] = [[] for _ in range(world)]
    for k in sorted(range(d), key=lambda k: (-w[k], k)):
        r = min(range(world), key=lambda r: (load[r], r))
        parts[r].append(k)
        load[r] += w[k]
    return [sorted(p) for p in parts]


def gather_limbs(compact: torch.Tensor, parts: list[list[int]], d: int, out: torch.Tensor | None = None):
    """All-gather every rank's output limbs and assemble them on every rank.

    compact: this rank's limbs, ``[B][len(parts[rank])][...]`` (slot s = limb parts[rank][s]).
    Returns ``[B][d][...]`` (written into ``out`` when given).  The collective moves each limb once
    per receiving rank; limbs are concatenated, never summed."""
    world = dist.get_world_size()
    B = compact.shape[0]
    tail = tuple(compact.shape[2:])
    m = max(len(p) for p in parts)
    if compact.shape[1] == m:
        pad = compact.contiguous()
    else:
        pad = torch.zeros((B, m) + tail, dtype=compact.dtype, device=compact.device)
        pad[:, : compact.shape[1]] = compact
    got = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(got, pad)
    if out is None:
        out = torch.empty((B, d) + tail, dtype=compact.dtype, device=compact.device)
    for r, ls in enumerate(parts):
        if ls:
            out[:, ls] = got[r][:, : len(ls)]
    return out


def split_plan(B: int, d: int, world: int, weights=None):
    """2-D partition of ONE dbfv_mul batch (B items, d output limbs) over ``world`` ranks: P_b item
    blocks x P_l limb groups, P_b P_l = world.  Rank r = ib * P_l + il computes the items
    ``shard(B, ib, P_b)`` and the output limbs ``limb_partition(d, P_l, weights)[il]`` (whole limbs:
    no cross-GPU sum, dbfv/eval.rs:109-132).  The factorisation taken is the one with no idle rank and
    the smallest largest per-rank product count; ties go to fewer limb groups (a chain then needs no
    exchange between its steps: every rank keeps whole items).  Only when every factorisation leaves
    a rank idle (B P_l < world for all P_l <= d, e.g. a single dbfv_mul on more ranks than limbs) is
    the least-idle one taken.  Deterministic: every rank computes the same plan without communicating.

    Returns (plan, P_b, P_l) with plan[r] = (item_start, item_count, limbs)."""
    w = limb_products(d) if weights is None else list(weights)
    best = None
    for pl in range(1, world + 1):
        if world % pl:
            continue
        pb = world // pl
        parts = limb_partition(d, pl, w)
        plan = []
        for r in range(world):
            ib, il = divmod(r, pl)
            s0, cnt = shard(B, ib, pb)
            plan.append((s0, cnt, parts[il]))
        loads = [cnt * sum(w[k] for k in ls) for _, cnt, ls in plan]
        idle = sum(1 for (_, cnt, ls) in plan if cnt == 0 or not ls)
        key = (idle, max(loads), pl)
        if best is None or key < best[0]:
            best = (key, plan, pb, pl)
    return best[1], best[2], best[3]


def gather_plan(compact: torch.Tensor, plan, rank: int, d: int, allgather, out: torch.Tensor):
    """Assemble every rank's part of a split dbfv_mul on every rank.

    compact: this rank's ``[item_count][len(limbs)][...]`` block (slot s = limb limbs[s]).  ``allgather(send,
    recv)`` fills recv ``[world][...send.shape]`` with every rank's send block (the library's
    ``exacto_rccl_allgather_u64`` on the GPU, torch.distributed on CPU): limbs are concatenated and
    placed, never summed (an RCCL sum of residues would overflow mod q).  Blocks are padded to the
    largest (items, limbs) block of the plan.  Writes ``out`` = ``[B][d][...]``."""
    mi = max(c for _, c, _ in plan)
    ml = max(len(ls) for _, _, ls in plan)
    tail = tuple(compact.shape[2:])
    _, cnt, ls = plan[rank]
    if tuple(compact.shape[:2]) == (mi, ml) and compact.is_contiguous():
        pad = compact
    else:
        pad = torch.zeros((mi, ml) + tail, dtype=compact.dtype, device=compact.device)
        pad[:cnt, : len(ls)] = compact[:cnt, : len(ls)]
    recv = torch.empty((len(plan), mi, ml) + tail, dtype=compact.dtype, device=compact.device)
    allgather(pad, recv)
    for r, (s0, c, lr) in enumerate(plan):
        if c and lr:
            if len(lr) == d and lr == list(range(d)):
                out[s0:s0 + c] = recv[r, :c, :d]
            else:
                out[s0:s0 + c, lr] = recv[r, :c, : len(lr)]
    return out


def torch_allgather(send: torch.Tensor, recv: torch.Tensor):
    """allgather for gather_plan over the default torch.distributed group (gloo or nccl)."""
    dist.all_gather(list(recv.unbind(0)), send)

