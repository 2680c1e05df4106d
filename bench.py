#!/usr/bin/env python3
"""Benchmark of the MI355X ciphertext-multiplication path (BASELINE.json metric).

Workload (default, BASELINE configs[2]): bfv_mul_and_relin at n=4096, 3x60-bit RNS limbs,
p=65537, gadget base 2^16 (G=12), a batch of 1024 independent ciphertext pairs per GPU
(weak scaling).  Synthetic data: uniform canonical residues per limb (the path is deterministic
given (ct1, ct2, rlk), so encrypted vs uniform inputs cost the same), resident in HBM before the
timed region starts.

A step is `reps` passes of the hot path, each over one whole batch (the input batches rotate over
two resident copies).  `reps` is chosen after the warm-up so that the K timed steps last at least
--min-time seconds (default 3 s: the batch-count estimate comes from two untimed batches and reads
high by up to ~35 %, so the region itself lands at >= 2 s): the BASELINE batch (1024 products, ~2.5 ms) is far shorter than
anything a wall-clock or GPU-busy sampler can see.  value = units processed / timed seconds.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` (N > 1, no WORLD_SIZE in the
environment) starts `torch.distributed.run --nproc-per-node N` on itself as a CHILD process, before
touching any GPU, and exits with its status; under torchrun WORLD_SIZE must equal --gpus.
  --split batch (default): every rank processes its own batch shard, no data-path collective; the
      relinearisation key is made on rank 0 and broadcast by the library's RCCL (ncclBroadcast into
      each rank's resident key).  value = total units over all ranks / max-over-ranks time (weak).
  --split limbs (dBFV configs): ONE dbfv_mul batch of B items split over the ranks in two dimensions
      (exacto_amd.dist.split_plan): P_b item blocks x P_l output-limb groups, P_b P_l = N, the
      factorisation with no idle rank and the smallest per-rank product count (limb k sums the pairs
      i + j = k, dbfv/eval.rs:109-132, so whole limbs need no cross-GPU sum).  Each rank computes its
      block, then the library's exacto_rccl_allgather_u64 assembles every item and limb on every
      rank (with P_l = 1 a chain runs locally and gathers once; with P_l > 1 after every step).
      value = B units / max-over-ranks time (strong scaling: the total work is fixed).
  --dry: no HIP calls at all (gloo on CPU, a stand-in step on CPU tensors of the same shapes): checks
      the launcher, the sharding / limb partition + gather and the timing path on a machine without
      a GPU.  Its numbers measure nothing.

Also reported on the same JSON line:
  roofline     — the kernel family with the largest share of one profiled batch (HIP events around
                 each of its launches, on the stream it runs on), its ALGORITHMIC bytes per launch
                 (each operand read once, each result written once) over its average
                 launch time, vs the 8 TB/s HBM peak; `ntt` = the same for the forward NTT, and
                 `kernels` the whole profiled breakdown;
  cpu_baseline — the C restatement of the reference algorithm (oracle/c: exact BigInt schoolbook
                 tensor, eval.rs:113-147; dbfv_mul with all d^2 products) on a bounded sample of the
                 same workload, on the host cores, rank 0 at N=1 only.
"""

from __future__ import annotations

import argparse
import datetime
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]
Q4 = Q3 + [1152921504606601217]
HBM_PEAK_GBS = 8000.0

# name: (n, moduli, aux, BFV plain modulus, gadget base, dBFV (d, base, p) or None, chain depth)
CONFIGS = {
    # BASELINE configs[0] = compact_bfv (presets.rs:24-35): the literal HPS multiplier with one aux
    # prime, G = 3; the configuration of the reference's published ~390 us (README.md:153)
    "cfg1": (1024, [1099509805057], [562949953443841], 257, 1 << 16, None, 0),
    "cfg2": (4096, [1152921504606830593], [], 65537, 1 << 16, None, 0),   # NTT fwd + mul + inv
    "cfg3": (4096, Q3, [], 65537, 1 << 16, None, 0),                      # bfv_mul_and_relin
    "cfg4": (4096, Q3, [], 260111, 1 << 16, (2, 256, 65536), 1),          # dbfv_mul
    "cfg5": (8192, Q4, [], 1040407, 256, (8, 256, 0), 4),                 # dbfv_mul chain depth 4
    # SURVEY 8(f) rank 4 (widened row, not a BASELINE config): Galois key switching
    # bfv_apply_automorphism (eval.rs:512-561) on cfg3's parameters, element 5
    "galois": (4096, Q3, [], 65537, 1 << 16, None, 0),
    # u64_dbfv (presets.rs:61-75), the profile of the reference's published dbfv_mul 31.395 ms
    # (reports/paper_reproduction.md:9, src/bin/paper_repro.rs:84-95): n = 4096, one 60-bit q, two
    # HPS aux primes, t = 1040407, gadget 256 (G = 8), d = 8, b = 256, p = 2^64
    "u64dbfv": (4096, [1152921504606830593], [18014398509998081, 36028797018972161], 1040407, 256,
                (8, 256, 0), 1),
}
DEFAULT_BATCH = {"cfg1": 8192, "cfg2": 16384, "cfg3": 1024, "cfg4": 1024, "cfg5": 8, "galois": 1024,
                 "u64dbfv": 64}
# the reference's own published numbers for a configuration (CPU, hardware unstated): one call's latency
PUBLISHED = {
    "cfg1": {"op": "bfv_mul_and_relin", "latency_us": 390.0, "source": "README.md:153 (compact_bfv)"},
    "u64dbfv": {"op": "dbfv_mul", "latency_us": 31395.0,
                "source": "reports/paper_reproduction.md:9 (d=8, b=2^8, u64_dbfv)"},
}

# profiled kernel families (exacto_hip.h exacto_prof_read kinds, context.hip ProfKind)
KINDS = {0: "fwd_ntt", 1: "inv_ntt", 2: "tensor_inv", 3: "polymul", 4: "exact_lift", 5: "exact_scale",
         6: "ks32_digit_ntt", 7: "ks32_mac", 8: "ks32_crt", 9: "dbfv_pairsum", 10: "psum_scale",
         12: "ks32_digit_sum", 13: "dbfv_combine", 14: "hps_extend", 15: "relin_mac",
         16: "hps_scale"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="work items per GPU (0 = config default)")
    ap.add_argument("--chunk", type=int, default=0, help="products per pipeline chunk (0 = library default)")
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--split", default="batch", choices=("batch", "limbs"))
    ap.add_argument("--min-time", type=float, default=3.0, help="lower bound of the timed region, seconds")
    ap.add_argument("--reps", type=int, default=0, help="batches per step (0 = from --min-time)")
    ap.add_argument("--dry", action="store_true", help="no HIP calls: CPU/gloo stand-in of the step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the batch-1 latency block (PMC passes: only full-batch dispatches)")
    ap.add_argument("--cpu-sample", type=int, default=0, help="units timed for the CPU baseline (0 = auto)")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch(args) -> int:
    """--gpus N > 1 outside torchrun: run torchrun on this script as a child (no exec: the parent
    has not touched the GPU and only waits), return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def _entry(rec, name, share=None):
    ms, nl, by = rec["ms"], max(rec["launches"], 1), rec["bytes"]
    achieved = by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    e = {"kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "launches": rec["launches"],
         "avg_launch_us": round(ms * 1000.0 / nl, 2), "bytes_per_launch": by / nl}
    if share is not None:
        e["share_of_profiled_batch"] = round(share, 4)
    return e


def _latest_profile(suffix):
    """profiles/rN_<suffix> of the latest round that has one (the committed PMC passes), or None."""
    for r in range(9, 0, -1):
        f = os.path.join(ROOT, "profiles", f"r{r}_{suffix}")
        if os.path.exists(f):
            return f
    return None


def roofline_block(ctx, step_one, cfg, n, L, S, batches=3):
    """`batches` profiled batches after the timed region (single lane: per-kernel events time each
    kernel alone), every family; launch averages over all of them."""
    import torch
    ctx.prof_enable(True)
    for _ in range(batches):
        step_one()
    torch.cuda.synchronize()
    recs = {k: ctx.prof_read(k) for k in KINDS}
    # what actually ran, as the library recorded it at launch (exacto_prof_kernels: the rocprofv3 names)
    ran = {k: ctx.prof_kernels(k) for k in KINDS}
    ctx.prof_enable(False)
    names = {k: " + ".join(nm for nm, _, _ in v) for k, v in ran.items() if v}
    total = sum(r["ms"] for r in recs.values())
    table = {KINDS[k]: _entry(r, names.get(k, KINDS[k]), r["ms"] / total if total else 0.0)
             for k, r in recs.items() if r["launches"]}
    top = max(recs, key=lambda k: recs[k]["ms"])
    roof = {"bound": "hbm"}
    roof.update(_entry(recs[top], names.get(top, KINDS[top]), recs[top]["ms"] / total if total else 0.0))
    roof["family"] = KINDS[top]
    roof["traffic"] = None
    # HBM bytes per launch from the committed PMC passes over this bench configuration
    # (tools/pmc_traffic.sh: 2*FETCH_SIZE + WRITE_SIZE per dispatch with the gfx950 corrections)
    top_kernel = roof["kernel"].split(" + ")[0]
    tfile = _latest_profile(f"{cfg}_traffic.json")
    if tfile:
        with open(tfile) as f:
            tr = json.load(f).get("kernels", {})
        hit = [v for k, v in tr.items() if k == top_kernel] or \
              [v for k, v in tr.items() if top_kernel.split("<")[0] in k]
        if hit:
            roof["traffic"] = round(hit[0]["traffic_bytes_avg"], 1)
            roof["traffic_over_algorithmic"] = round(hit[0]["traffic_bytes_avg"] / roof["bytes_per_launch"], 4)
            roof["traffic_source"] = os.path.relpath(tfile, ROOT)
    # the compute-side ceiling (integer modular arithmetic: VALU issue, not MFMA) from the committed
    # PMC pass: VALU wave-instructions and GPU cycles per dispatch, ~4.4 cycles per integer
    # multiply-class wave-instruction per SIMD (tools/op_rate.hip), 1024 SIMDs
    vfile = _latest_profile(f"{cfg}_valu_counters.json")
    if vfile:
        with open(vfile) as f:
            vc = json.load(f).get("kernels", {})
        hit = [v for k, v in vc.items() if k == top_kernel] or \
              [v for k, v in vc.items() if top_kernel.split("<")[0] in k]
        if hit:
            v = hit[0]
            need = v["valu_insts"] * 4.4 / 1024.0
            roof["compute"] = {"bound": "valu", "valu_insts_per_launch": round(v["valu_insts"]),
                               "cycles_per_valu": 4.4, "gpu_cycles_per_launch": round(v["gpu_cycles"]),
                               "frac": round(need / v["gpu_cycles"], 3), "source": os.path.relpath(vfile, ROOT)}
    ntt = table.get("fwd_ntt")
    return roof, ntt, table


def _rate(run, threads, target_s, cap):
    """units/s of run(k, threads): one unit per thread first, then (when that took well under the
    target) a sample sized to about target_s seconds.  Returns (rate, units, seconds)."""
    k = threads
    t0 = time.perf_counter()
    run(k, threads)
    dt = time.perf_counter() - t0
    if dt < 0.25 * target_s and k < cap:
        k = min(cap, max(k, int(k * target_s / max(dt, 1e-6)) // threads * threads))
        t0 = time.perf_counter()
        run(k, threads)
        dt = time.perf_counter() - t0
    return k / dt, k, dt


def cpu_baseline(cfg, n, moduli, aux, plain, gbase, dbfv, depth, sample):
    """The C restatement of the reference algorithm (oracle/c) on a bounded sample of the workload,
    timed on the host cores this job may use (16 on the GPU box, whose os.cpu_count() reports the
    whole machine) and on one thread.  OpenMP over the products mirrors the reference's rayon fan-out
    of dbfv_mul's d^2 products (dbfv/eval.rs:117-122).  Each unit is the whole reference operation:
    a bfv_mul_and_relin (HPS for cfg1 / u64dbfv, the exact BigInt schoolbook tensor otherwise,
    eval.rs:89-413), a dbfv_mul item with all d^2 products, or cfg2's NTT product (ntt.rs:181-195)."""
    import numpy as np
    from oracle import params as P, cref
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from bridge import uniform_residues
    if not cref.available():
        return {"value": None, "error": "oracle/c/liboracle.so not built"}
    threads = min(16, os.cpu_count() or 1)
    rng = np.random.default_rng(7)
    impl = "oracle/c (C restatement of the reference algorithm)"
    target_m, target_1 = 8.0, 4.0
    if cfg == "cfg2":
        q = moduli[0]
        pool = 4096
        a = rng.integers(0, q, size=(pool, n), dtype=np.uint64)
        b = rng.integers(0, q, size=(pool, n), dtype=np.uint64)

        def run(k, th):
            for s0 in range(0, k, pool):
                m = min(pool, k - s0)
                cref.polymul(n, q, a[:m], b[:m], threads=th)
        unit, what = "poly_mul/s", f"negacyclic NTT products (fwd x2 + pointwise + inv, n={n}, 1x60-bit)"
        cap = 1 << 22
    else:
        bld = P.BfvParamsBuilder().ring_degree(n).plain_modulus(plain).ct_moduli(moduli).gadget_base(gbase)
        if aux:
            bld = bld.aux_moduli(aux)
        prm = bld.build()
        rlk = uniform_residues(rng, (prm.gadget_digits, 2), moduli, n)
        pool = 64
        if dbfv is None or (depth > 1 and cfg == "cfg5"):
            ct1 = uniform_residues(rng, (pool, 2), moduli, n)
            ct2 = uniform_residues(rng, (pool, 2), moduli, n)

            def run_products(k, th):
                for s0 in range(0, k, pool):
                    m = min(pool, k - s0)
                    cref.bfv_mul_and_relin(prm, ct1[:m], ct2[:m], rlk, threads=th)
        if dbfv is None:
            run = run_products
            unit = "bfv_mul_and_relin/s"
            what = (f"bfv_mul_and_relin (n={n}, L={len(moduli)}, "
                    + ("literal HPS, eval.rs:157-413" if aux else "exact BigInt schoolbook tensor, eval.rs:113-147")
                    + f", G={prm.gadget_digits})")
            cap = 1 << 20
        else:
            d, base, dplain = dbfv
            dp = P.DbfvParams(prm, base, d, dplain)
            items = 1 if cfg == "cfg5" else 16
            xa = uniform_residues(rng, (items, d, 2), moduli, n)
            xb = uniform_residues(rng, (items, d, 2), moduli, n)

            def run(k, th):
                for s0 in range(0, k, items):
                    m = min(items, k - s0)
                    cref.dbfv_mul(dp, xa[:m], xb[:m], rlk, threads=th)
            unit = "dbfv_mul/s" if depth == 1 else f"dbfv_mul_chain(depth {depth})/s"
            what = f"dbfv_mul items (d={d}, all {d * d} products each, n={n}, L={len(moduli)}" + \
                   (", HPS products" if aux else "") + ")"
            cap = 1 << 16
            if cfg == "cfg5":
                # one measured dbfv_mul item (64 products, minutes on one thread at n = 8192), the chain
                # being `depth` identical dbfv_mul steps; one thread: single products x d^2
                t0 = time.perf_counter()
                run(1, threads)
                dt = time.perf_counter() - t0
                r1, k1, t1 = _rate(run_products, 1, target_1, 1 << 10)
                return {"value": 1.0 / dt / depth, "unit": unit, "cores": threads, "kind": "port",
                        "sample": f"one dbfv_mul item (d={d}: all {d * d} products, n={n}, L={len(moduli)}) in "
                                  f"{dt:.2f} s on {threads} threads, divided by the chain's {depth} steps; {impl}",
                        "single_thread": {"value": r1 / (d * d * depth), "cores": 1,
                                          "sample": f"{k1} bfv_mul_and_relin of the chain's parameters in {t1:.2f} s, "
                                                    f"/ {d * d * depth} products per chain"}}
    rm, km, tm = _rate(run, threads, target_m, cap)
    r1, k1, t1 = _rate(run, 1, target_1, cap)
    if depth > 1:
        rm, r1 = rm / depth, r1 / depth
    return {"value": rm, "unit": unit, "cores": threads, "kind": "port",
            "sample": f"{km} {what} in {tm:.2f} s on {threads} threads; {impl}",
            "single_thread": {"value": r1, "cores": 1, "sample": f"{k1} in {t1:.2f} s on 1 thread",
                              "us_per_unit": round(1e6 / r1, 1)}}


def latency_block(one_single, sync, reps=30):
    """One call of the path on one unit (batch 1: a single bfv_mul_and_relin / dbfv_mul / chain),
    synchronised, median over `reps` calls: the quantity the reference publishes (one call's latency
    on its CPU, README.md:153, reports/paper_reproduction.md:9)."""
    ts = []
    for _ in range(3):
        one_single()
    sync()
    for _ in range(reps):
        t0 = time.perf_counter()
        one_single()
        sync()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return {"median_us": round(1e6 * ts[len(ts) // 2], 1), "min_us": round(1e6 * ts[0], 1), "calls": reps,
            "batch": 1}


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(relaunch(args))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np  # noqa: F401
    import torch
    import torch.distributed as dist
    from exacto_amd import dist as xdist

    n, moduli, aux, plain, gbase, dbfv, depth = CONFIGS[args.config]
    L = len(moduli)
    B = args.batch or DEFAULT_BATCH[args.config]
    if args.split == "limbs" and dbfv is None:
        print("bench.py: --split limbs needs a dBFV config (cfg4, cfg5, u64dbfv)", file=sys.stderr)
        sys.exit(2)
    distributed = world > 1
    # deadline per phase of a multi-rank run: a rank that never joins a collective ends the job with a
    # diagnostic line instead of blocking it until the driver's time limit (exacto_amd.dist.Watchdog;
    # torch.distributed's own timeout and the library's RCCL deadlines, EXACTO_RCCL_TIMEOUT_S, likewise)
    wd = xdist.Watchdog(rank, enabled=distributed, withhold_ok=args.dry)
    # (torch's own collective timeout a minute later: the watchdog names the phase first)
    pg_timeout = datetime.timedelta(seconds=xdist.deadline_s() + 60.0)
    if distributed:
        wd.arm("init")
    if args.dry:
        device = torch.device("cpu")
        if distributed:
            dist.init_process_group("gloo", timeout=pg_timeout)
    else:
        if distributed:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)
    backend = dist.get_backend() if distributed else None

    def sync():
        if not args.dry:
            torch.cuda.synchronize(device)

    ctx = None
    G = None
    S = 0
    if not args.dry:
        from exacto_amd._ffi import HipContext
        ctx = HipContext(n, moduli, aux, plain, gbase, device=local)
        ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
        if args.chunk:
            ctx.set_chunk(args.chunk)
        G, S = ctx.G, ctx.ks32_primes
    else:   # compute_gadget_digits (params/mod.rs:126-140): the fewest g with base^g >= Q
        Q, G = math.prod(moduli), 0
        while gbase ** G < Q:
            G += 1

    gen = torch.Generator(device=device)
    gen.manual_seed(0xE7AC7003 + (rank if args.split == "batch" else 0))

    def uniform(shape_prefix, g=None):
        out = torch.empty(tuple(shape_prefix) + (L, n), dtype=torch.int64, device=device)
        for i, q in enumerate(moduli):
            out[..., i, :] = torch.randint(0, q, tuple(shape_prefix) + (n,), generator=g or gen, dtype=torch.int64,
                                           device=device)
        return out

    # relinearisation key: made on rank 0 only, broadcast by the library's RCCL into every rank's
    # resident key (ncclBroadcast over xGMI)
    key_collective = None
    comm, rccl_nranks = None, None
    if distributed:
        wd.arm("comm_init" if not args.dry else "key_broadcast")
    if distributed and not args.dry:
        # the library's own RCCL communicator; ncclCommCount on the line shows RCCL spans every rank
        comm = xdist.rccl_comm_for(ctx, local)
        rccl_nranks = comm.count()
        wd.arm("key_broadcast")
    if args.config != "cfg2":
        kgen = torch.Generator(device=device)
        kgen.manual_seed(0xE7AC7003)
        if args.dry:
            rlk = uniform((G, 2), kgen) if rank == 0 else torch.zeros((G, 2, L, n), dtype=torch.int64)
            if distributed:
                dist.broadcast(rlk, src=0)
                key_collective = "torch.distributed.broadcast (gloo, dry)"
        else:
            if rank == 0:
                rlk = uniform((G, 2), kgen)
                sync()
                ctx.load_relin_key_dev(rlk, G)
            if distributed:
                ctx.broadcast_relin_key(comm, 0, G)
                ctx.rccl_sync(comm)   # the broadcast's completion, with the library's deadline
                key_collective = "exacto_ctx_broadcast_relin_key (ncclBroadcast, library RCCL communicator)"
            sync()

    # ---- the step: one pass over one batch (`one(i)`, i = input copy), timed `reps` times per step
    nbuf = 2
    parts = None
    one_single = None   # one call on one unit (latency_block)
    if args.config == "cfg2":
        a = [uniform((B,)) for _ in range(nbuf)]
        b = [uniform((B,)) for _ in range(nbuf)]
        outs = [torch.empty_like(a[0]) for _ in range(nbuf)]
        mode = os.environ.get("EXACTO_BENCH_CFG2", "polymul")

        def one(i):   # fwd NTT of both operands, pointwise product, inverse NTT
            if args.dry:
                torch.add(a[i], b[i], out=outs[i])
            elif mode == "polymul":
                ctx.rns_polymul_dev(a[i], b[i], outs[i], B)
            else:
                outs[i].copy_(a[i])
                ctx.rns_fwd_dev(outs[i], B)
                ctx.rns_fwd_dev(b[i], B)
                if mode == "mulinv":
                    ctx.rns_mul_inv_dev(outs[i], b[i], outs[i], B)
                else:
                    ctx.rns_mul_dev(outs[i], b[i], outs[i], B)
                    ctx.rns_inv_dev(outs[i], B)
        unit = "poly_mul/s"
        metric = "NTT-based negacyclic poly muls/sec (fwd NTT x2 + pointwise + inv NTT)"
    elif args.config == "galois":
        ct = [uniform((B, 2)) for _ in range(nbuf)]
        gk = uniform((G, 2))
        outs = [torch.empty_like(ct[0]) for _ in range(nbuf)]

        def one(i):
            if args.dry:
                torch.add(ct[i], 1, out=outs[i])
            else:
                ctx.bfv_apply_automorphism_dev(ct[i], 5, gk, G, outs[i], B)
        unit = "bfv_apply_automorphism/s"
        metric = "Galois automorphisms/sec (bfv_apply_automorphism, key switched)"
    elif dbfv is None:
        ct1 = [uniform((B, 2)) for _ in range(nbuf)]
        ct2 = [uniform((B, 2)) for _ in range(nbuf)]
        outs = [torch.empty_like(ct1[0]) for _ in range(nbuf)]

        def one(i):
            if args.dry:
                torch.add(ct1[i], ct2[i], out=outs[i])
            else:
                ctx.bfv_mul_and_relin_dev(ct1[i], ct2[i], outs[i], B)

        def one_single():
            ctx.bfv_mul_and_relin_dev(ct1[0], ct2[0], outs[0], 1)
        unit = "bfv_mul_and_relin/s"
        metric = "ciphertext muls/sec (bfv_mul_and_relin)"
    else:
        d, base, dplain = dbfv
        x = [uniform((B, d, 2)) for _ in range(nbuf)]
        y = [uniform((B, d, 2)) for _ in range(nbuf)]
        outs = [torch.empty_like(x[0]) for _ in range(nbuf)]
        if args.split == "limbs":
            # ONE dbfv_mul batch over all ranks, 2-D: item blocks x output-limb groups (split_plan)
            wts = xdist.limb_products(d, base, dplain)
            plan, pb, pl = xdist.split_plan(B, d, world, wts) if distributed else ([(0, B, list(range(d)))], 1, 1)
            parts = {"item_blocks": pb, "limb_groups": pl, "ranks": [[c, ls] for _, c, ls in plan]}
            s0, cnt, mine = plan[rank]
            full = mine == list(range(d))
            compact = torch.zeros((max(cnt, 1), max(len(mine), 1), 2, L, n), dtype=torch.int64, device=device)
            acc = [torch.empty_like(x[0]), torch.empty_like(x[0])]
            if distributed and not args.dry:
                allgather = lambda snd, rcv: ctx.allgather_u64(comm, snd, rcv, snd.numel())
            else:
                allgather = xdist.torch_allgather

            def part_mul(src, yy, dst, steps):
                # this rank's items and limbs: `steps` chain steps when it holds whole items, else one
                if cnt and mine:
                    xs, ys = src[s0:s0 + cnt], yy[s0:s0 + cnt]
                    if args.dry:   # stand-in: limb k <- src[:, k] + steps * yy[:, k] (checks the gather)
                        torch.add(xs[:, mine], ys[:, mine], alpha=steps, out=compact[:cnt, : len(mine)])
                    elif full and steps > 1:
                        ctx.dbfv_mul_chain_dev(d, base, dplain, xs, ys, compact, cnt, steps)
                    elif full:
                        ctx.dbfv_mul_dev(d, base, dplain, xs, ys, compact, cnt)
                    else:
                        ctx.dbfv_mul_limbs_dev(d, base, dplain, xs, ys, compact, cnt, mine)
                if distributed:
                    xdist.gather_plan(compact[:cnt, : len(mine)], plan, rank, d, allgather, dst)
                else:
                    dst.copy_(compact)

            def one(i):
                # depth-`depth` chain (paper_repro semantics, src/bin/paper_repro.rs:155-158, 217-220);
                # whole items per rank (P_l = 1): the chain runs locally, one gather at the end
                if pl == 1:
                    part_mul(x[i], y[i], outs[i], depth)
                    return
                src = x[i]
                for st in range(depth):
                    dst = outs[i] if st == depth - 1 else acc[st % 2]
                    part_mul(src, y[i], dst, 1)
                    src = dst
        else:
            def one(i):
                # depth-`depth` chain: acc <- dbfv_mul(acc, y), mul_depth reset before every step
                # (paper_repro semantics, src/bin/paper_repro.rs:155-158, 217-220), one native call
                if args.dry:
                    torch.add(x[i], y[i], out=outs[i])
                elif depth == 1:
                    ctx.dbfv_mul_dev(d, base, dplain, x[i], y[i], outs[i], B)
                else:
                    ctx.dbfv_mul_chain_dev(d, base, dplain, x[i], y[i], outs[i], B, depth)

            def one_single():
                if depth == 1:
                    ctx.dbfv_mul_dev(d, base, dplain, x[0], y[0], outs[0], 1)
                else:
                    ctx.dbfv_mul_chain_dev(d, base, dplain, x[0], y[0], outs[0], 1, depth)
        unit = "dbfv_mul/s" if depth == 1 else f"dbfv_mul_chain(depth {depth})/s"
        metric = "ciphertext muls/sec (dbfv_mul)" if depth == 1 else f"dbfv_mul chains/sec (depth {depth})"
    sync()

    if distributed:
        wd.arm("warmup")
    for w in range(args.warmup):
        one(w % nbuf)
    sync()
    # batches per step: the K timed steps last >= --min-time (the slowest rank decides)
    reps = args.reps
    per = 0.0
    if reps <= 0:
        t0 = time.perf_counter()
        for i in range(nbuf):
            one(i)
        sync()
        per = (time.perf_counter() - t0) / nbuf
        per = xdist.max_over_ranks(per, device=device if backend == "nccl" else None)
        reps = max(1, math.ceil(args.min_time / max(args.steps * per, 1e-9)))

    def step():
        for r in range(reps):
            one(r % nbuf)

    if distributed:
        # the timed region: one deadline plus ten times its expected length
        wd.arm("timed", xdist.deadline_s() + 10.0 * args.steps * reps * per)
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    if distributed:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    elapsed = xdist.max_over_ranks(elapsed, device=device if backend == "nccl" else None)
    ms_per_step = 1000.0 * elapsed / args.steps
    units_per_step = B * reps
    total_units = (world if args.split == "batch" else 1) * units_per_step * args.steps
    value = total_units / elapsed
    if distributed:
        wd.arm("report")

    dry_check = None
    if args.dry and args.split == "limbs":
        # stand-in chain: every step adds y, so the assembled output is x + depth * y on every limb
        dry_check = bool(torch.equal(outs[(reps - 1) % nbuf], x[(reps - 1) % nbuf] + depth * y[(reps - 1) % nbuf]))

    roofline, ntt, kernels = None, None, None
    if not args.dry:
        roofline, ntt, kernels = roofline_block(ctx, lambda: one(0), args.config, n, L, S)

    latency = None
    if one_single is not None and not args.dry and world == 1 and not args.no_latency:
        latency = latency_block(one_single, sync)
        if args.config in PUBLISHED:
            pub = PUBLISHED[args.config]
            latency["reference_published_us"] = pub["latency_us"]
            latency["reference_source"] = pub["source"] + "; reference Rust CPU, hardware unstated"

    cpu = None
    if (rank == 0 and world == 1 and not args.dry and not args.no_cpu_baseline
            and args.config != "galois"):
        try:   # informative; never fail the bench on it
            cpu = cpu_baseline(args.config, n, moduli, aux, plain, gbase, dbfv, depth, args.cpu_sample)
        except Exception as e:
            cpu = {"value": None, "error": repr(e)}

    if rank == 0:
        workload = {"cfg1": "bfv_mul_and_relin on compact_bfv (n=1024, 40-bit q, 1 HPS aux prime, G=3), "
                            "BASELINE configs[0]",
                    "u64dbfv": "dbfv_mul on u64_dbfv (n=4096, 60-bit q + 2 HPS aux primes, d=8 b=256 p=2^64, "
                               "gadget 256), the reference's published paper_repro profile",
                    "cfg2": "batched fwd NTT + pointwise mul + inv NTT, BASELINE configs[1]",
                    "cfg3": "bfv_mul_and_relin, BASELINE configs[2]",
                    "cfg4": "dbfv_mul d=2 b=256 p=2^16, BASELINE configs[3]",
                    "cfg5": "dbfv_mul chain depth 4, d=8 b=256 p=2^64, BASELINE configs[4]",
                    "galois": "bfv_apply_automorphism (element 5, key switched) on cfg3 parameters, "
                              "SURVEY 8(f) rank 4"}[args.config]
        line = {
            "metric": metric,
            "value": round(value, 1),
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak" if args.split == "batch" else "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (uniform canonical residues per limb, seeded; two resident input copies "
                    "rotated; rlk made on rank 0 and broadcast)" + ("; DRY RUN: no GPU work" if args.dry else ""),
            "config": {"workload": workload, "ring_degree": n, "ct_limbs": L,
                       "limb_bits": max(q.bit_length() for q in moduli),
                       "aux_moduli": aux or None,
                       "plain_modulus": plain, "gadget_base": gbase, "gadget_digits": G,
                       "batch_per_gpu": B if args.split == "batch" else None,
                       "global_batch": B * (world if args.split == "batch" else 1),
                       "batches_per_step": reps, "units_per_step": units_per_step,
                       "parallelism": (f"batch-shard x{world}" if args.split == "batch"
                                       else f"one dbfv_mul batch split x{world}: {parts['item_blocks']} item "
                                            f"blocks x {parts['limb_groups']} output-limb groups"),
                       "split_plan": parts if args.split == "limbs" else None},
            "world_size": world,
            "backend": backend,
            "key_broadcast": key_collective,
            "rccl_nranks": rccl_nranks,
            "timed_s": round(elapsed, 3),
            "roofline": roofline,
            "ntt": ntt,
            "kernels": kernels,
            "cpu_baseline": cpu,
            "latency": latency,
        }
        if dbfv is not None:
            line["config"].update({"dbfv_digits": dbfv[0], "dbfv_base": dbfv[1],
                                   "dbfv_plain_modulus": dbfv[2] or "2^64", "chain_depth": depth})
        if args.dry:
            line["dry"] = True
            if dry_check is not None:
                line["dry_gather_ok"] = dry_check
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        if comm is not None:
            sync()
            comm.close()
        dist.destroy_process_group()
        wd.disarm()


if __name__ == "__main__":
    main()
