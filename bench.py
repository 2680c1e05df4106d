#!/usr/bin/env python3
"""Benchmark of the MI355X ciphertext-multiplication path (BASELINE.json metric).

Workload (default, BASELINE configs[2]): bfv_mul_and_relin at n=4096, 3x60-bit RNS limbs,
p=65537, gadget base 2^16 (G=12), a batch of 1024 independent ciphertext pairs per GPU
(weak scaling).  A "step" is one pass of the whole batch through the path, with inputs
already resident in HBM.  Synthetic data: uniform canonical residues per limb (the path
is deterministic given (ct1, ct2, rlk), so encrypted vs uniform inputs cost the same).

Multi-GPU: one process per GPU (torchrun).  The relinearisation key is generated on rank 0
and broadcast over RCCL (xGMI); every rank then processes its own batch shard with no
data-path collective.  value = total products over all ranks / max-over-ranks step time.

Also reported on the same JSON line:
  roofline     — the dominant kernel (forward NTT of the pipeline), algorithmic bytes
                 16*n per residue polynomial over its summed launch time,
                 measured with HIP events around each of its launches on the pipeline's
                 stream, vs the 8 TB/s HBM peak;
  cpu_baseline — the CPU restatement of the reference algorithm (oracle/, exact BigInt
                 schoolbook tensor, eval.rs:113-147) on a bounded sample, rank 0 at N=1.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from exacto_amd._ffi import HipContext  # noqa: E402

Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]
Q4 = Q3 + [1152921504606601217]
HBM_PEAK_GBS = 8000.0

# name: (n, moduli, aux, BFV plain modulus, gadget base, dBFV (d, base, p) or None, chain depth)
CONFIGS = {
    "cfg2": (4096, [1152921504606830593], [], 65537, 1 << 16, None, 0),   # NTT fwd + mul + inv
    "cfg3": (4096, Q3, [], 65537, 1 << 16, None, 0),                      # bfv_mul_and_relin
    "cfg4": (4096, Q3, [], 260111, 1 << 16, (2, 256, 65536), 1),          # dbfv_mul
    "cfg5": (8192, Q4, [], 1040407, 256, (8, 256, 0), 4),                 # dbfv_mul chain depth 4
    # SURVEY 8(f) rank 4 (widened row, not a BASELINE config): Galois key switching
    # bfv_apply_automorphism (eval.rs:512-561) on cfg3's parameters, element 5
    "galois": (4096, Q3, [], 65537, 1 << 16, None, 0),
}
DEFAULT_BATCH = {"cfg2": 16384, "cfg3": 1024, "cfg4": 1024, "cfg5": 8, "galois": 1024}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="work items per GPU (0 = config default)")
    ap.add_argument("--chunk", type=int, default=0, help="products per pipeline chunk (0 = library default)")
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="products timed for the CPU baseline (0 = auto)")
    return ap.parse_args()


def uniform_dev(shape_prefix, moduli, n, gen, device):
    out = torch.empty(tuple(shape_prefix) + (len(moduli), n), dtype=torch.int64, device=device)
    for i, q in enumerate(moduli):
        out[..., i, :] = torch.randint(0, q, tuple(shape_prefix) + (n,), generator=gen,
                                       dtype=torch.int64, device=device)
    return out


def cpu_baseline(n, moduli, plain, gbase, sample, threads=1):
    """Time the CPU restatement of the reference algorithm on `sample` products, batch-parallel
    over `threads` OpenMP threads (the reference fans dbfv_mul out over rayon the same way)."""
    from oracle import params as P
    from oracle import bfv as obfv
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from bridge import uniform_residues, np_to_ct, np_to_rlk
    try:
        from oracle import cref
        use_c = cref.available()
    except Exception:
        use_c = False
    prm = P.BfvParamsBuilder().ring_degree(n).plain_modulus(plain).ct_moduli(moduli).gadget_base(gbase).build()
    rng = np.random.default_rng(7)
    ct1 = uniform_residues(rng, (sample, 2), moduli, n)
    ct2 = uniform_residues(rng, (sample, 2), moduli, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), moduli, n)
    if use_c:
        t0 = time.perf_counter()
        cref.bfv_mul_and_relin(prm, ct1, ct2, rlk, threads=threads)
        dt = time.perf_counter() - t0
        impl = "oracle/c (C restatement, exact multiword schoolbook tensor)"
    else:
        threads = 1
        rk = np_to_rlk(rlk, prm)
        t0 = time.perf_counter()
        for b in range(sample):
            obfv.bfv_mul_and_relin(np_to_ct(ct1[b], prm), np_to_ct(ct2[b], prm), rk)
        dt = time.perf_counter() - t0
        impl = "oracle/ (Python exact-integer restatement)"
    return {"value": sample / dt, "unit": "bfv_mul_and_relin/s", "cores": threads, "kind": "port",
            "sample": f"{sample} bfv_mul_and_relin of the same workload (n={n}, L={len(moduli)}), "
                      f"{threads} thread(s), {impl}; {dt:.2f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    n, moduli, aux, plain, gbase, dbfv, depth = CONFIGS[args.config]
    L = len(moduli)
    B = args.batch or DEFAULT_BATCH[args.config]
    ctx = HipContext(n, moduli, aux, plain, gbase, device=local)
    stream = torch.cuda.current_stream(device)
    ctx.set_stream(stream.cuda_stream)
    if args.chunk:
        ctx.set_chunk(args.chunk)
    G = ctx.G

    gen = torch.Generator(device=device)
    gen.manual_seed(0xE7AC7003 + rank)
    kgen = torch.Generator(device=device)
    kgen.manual_seed(0xE7AC7003)
    if args.config == "cfg2":
        a = uniform_dev((B,), moduli, n, gen, device)
        b = uniform_dev((B,), moduli, n, gen, device)

        # EXACTO_BENCH_CFG2: "polymul" (default) one fused kernel per product (exacto_rns_polymul_dev);
        # "mulinv" forward transforms + product fused into the inverse; "unfused" the four API calls
        mode = os.environ.get("EXACTO_BENCH_CFG2", "polymul")

        def step():  # fwd NTT of both operands, pointwise product, inverse NTT
            if mode == "polymul":
                ctx.rns_polymul_dev(a, b, a, B)
                return
            ctx.rns_fwd_dev(a, B)
            ctx.rns_fwd_dev(b, B)
            if mode == "mulinv":
                ctx.rns_mul_inv_dev(a, b, a, B)
            else:
                ctx.rns_mul_dev(a, b, a, B)
                ctx.rns_inv_dev(a, B)
        units_per_step = B
        unit = "poly_mul/s"
        metric = "NTT-based negacyclic poly muls/sec (fwd NTT x2 + pointwise + inv NTT)"
    else:
        # relinearisation key: made once on rank 0, RCCL-broadcast to every GPU
        rlk = uniform_dev((G, 2), moduli, n, kgen, device) if rank == 0 else \
            torch.empty((G, 2, L, n), dtype=torch.int64, device=device)
        if distributed:
            dist.broadcast(rlk, src=0)
        torch.cuda.synchronize(device)
        ctx.load_relin_key_dev(rlk, G)
        if args.config == "galois":
            ct1 = uniform_dev((B, 2), moduli, n, gen, device)
            gk = uniform_dev((G, 2), moduli, n, kgen, device)
            out = torch.empty_like(ct1)

            def step():
                ctx.bfv_apply_automorphism_dev(ct1, 5, gk, G, out, B)
            units_per_step = B
            unit = "bfv_apply_automorphism/s"
            metric = "Galois automorphisms/sec (bfv_apply_automorphism, key switched)"
        elif dbfv is None:
            ct1 = uniform_dev((B, 2), moduli, n, gen, device)
            ct2 = uniform_dev((B, 2), moduli, n, gen, device)
            out = torch.empty_like(ct1)

            def step():
                ctx.bfv_mul_and_relin_dev(ct1, ct2, out, B)
            units_per_step = B
            unit = "bfv_mul_and_relin/s"
            metric = "ciphertext muls/sec (bfv_mul_and_relin)"
        else:
            d, base, dplain = dbfv
            x = uniform_dev((B, d, 2), moduli, n, gen, device)
            y = uniform_dev((B, d, 2), moduli, n, gen, device)
            bufs = [torch.empty_like(x), torch.empty_like(x)]

            def step():
                # depth-`depth` chain: acc <- dbfv_mul(acc, y), mul_depth reset before every step
                # (paper_repro semantics, src/bin/paper_repro.rs:155-158, 217-220), one native call
                if depth == 1:
                    ctx.dbfv_mul_dev(d, base, dplain, x, y, bufs[0], B)
                else:
                    ctx.dbfv_mul_chain_dev(d, base, dplain, x, y, bufs[0], B, depth)
            units_per_step = B
            unit = "dbfv_mul/s" if depth == 1 else f"dbfv_mul_chain(depth {depth})/s"
            metric = "ciphertext muls/sec (dbfv_mul)" if depth == 1 else \
                f"dbfv_mul chains/sec (depth {depth})"
    torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * units_per_step * args.steps / elapsed

    # roofline of the dominant kernel: one profiled step, HIP events around every NTT launch
    ctx.prof_enable(True)
    step()
    torch.cuda.synchronize(device)
    fwd = ctx.prof_read(0)
    inv = ctx.prof_read(1)
    fused = ctx.prof_read(3)
    ctx.prof_enable(False)
    logn = n.bit_length() - 1
    # every BASELINE prime lies in (2^60 - 2^32, 2^60): n = 4096 / 8192 take the hand-scheduled
    # kernels (n = 4096 forward: the persistent LDS-DMA form)
    on = lambda k: os.environ.get(k, "1") != "0"
    asm = logn in (12, 13) and on("EXACTO_NTT_ASM")
    fwd_name = ("ntt_fwd_pipe_kernel" if asm and logn == 12 and on("EXACTO_NTT_PIPE")
                else f"ntt_fwd_asm_kernel<{logn}>" if asm else f"ntt_fwd_kernel<{logn}>")
    inv_name = f"ntt_inv_asm_kernel<{logn}>" if asm and on("EXACTO_NTT_ASM_INV") else f"ntt_inv_kernel<{logn}>"
    dom, dom_name = (fwd, fwd_name) if fwd["ms"] >= inv["ms"] else (inv, inv_name)
    if fused["ms"] > dom["ms"]:   # cfg2's fused product kernel (3 transforms; bytes: a, b in, product out)
        dom, dom_name = fused, f"ntt_polymul_kernel<{logn}>"
    achieved = dom["bytes"] / (dom["ms"] * 1e-3) / 1e9 if dom["ms"] > 0 else 0.0
    per_launch_ms = dom["ms"] / max(dom["launches"], 1)
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None,
        "kernel": dom_name,
        "launches_per_step": dom["launches"],
        "avg_launch_us": round(per_launch_ms * 1000.0, 2),
        "bytes_per_launch": dom["bytes"] / max(dom["launches"], 1),
        "polys_per_step": dom["polys"],
        "ntt_share_of_step": round((fwd["ms"] + inv["ms"] + fused["ms"]) / ms_per_step, 3),
    }
    # HBM bytes per launch from the committed PMC passes over this same bench configuration
    # (tools/pmc_traffic.sh: 2*FETCH_SIZE + WRITE_SIZE per dispatch, gfx950 corrections, averaged
    # over every forward-NTT dispatch: the same launch mix per step as the timed one)
    tfile = os.path.join(ROOT, "profiles", f"r2_{args.config}_fwd_traffic.json")
    if dom_name.startswith("ntt_fwd") and os.path.exists(tfile):
        with open(tfile) as f:
            tr = json.load(f)
        roofline["traffic"] = round(tr["traffic_bytes_avg"], 1)
        roofline["traffic_over_algorithmic"] = round(tr["traffic_bytes_avg"] / roofline["bytes_per_launch"], 4)
        roofline["traffic_source"] = os.path.relpath(tfile, ROOT)

    # the compute-side ceiling of the same kernel (integer modular arithmetic: the VALU issue rate,
    # not MFMA): VALU wave-instructions and GPU cycles per dispatch from the committed PMC pass
    # over this bench (tools/r2_evidence.sh), at the measured ~4.4 cycles per integer
    # multiply-class wave-instruction per SIMD (tools/op_rate.hip, 1024 SIMDs)
    vfile = os.path.join(ROOT, "profiles", f"r2_{args.config}_valu_counters.json")
    if os.path.exists(vfile):
        with open(vfile) as f:
            vc = json.load(f)["kernels"]
        hit = [v for k, v in vc.items() if dom_name.split("<")[0] in k]
        if hit:
            v = hit[0]
            need = v["valu_insts"] * 4.4 / 1024.0
            roofline["compute"] = {"bound": "valu", "valu_insts_per_launch": round(v["valu_insts"]),
                                   "cycles_per_valu": 4.4, "gpu_cycles_per_launch": round(v["gpu_cycles"]),
                                   "frac": round(need / v["gpu_cycles"], 3),
                                   "source": os.path.relpath(vfile, ROOT)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "cfg3":
        # all the host cores this job may use (16 on the GPU box, whose os.cpu_count() reports the
        # whole machine), one product per thread; the single-thread figure rides along
        threads = min(16, os.cpu_count() or 1)
        try:
            # about 10-15 s of CPU work: 8 products per thread
            cpu = cpu_baseline(n, moduli, plain, gbase, args.cpu_sample or 8 * threads, threads)
            one = cpu_baseline(n, moduli, plain, gbase, 2, 1)
            cpu["single_thread"] = {"value": one["value"], "sample": one["sample"]}
        except Exception as e:  # the baseline is informative; never fail the bench on it
            cpu = {"value": None, "error": repr(e)}

    if rank == 0:
        workload = {"cfg2": "batched fwd NTT + pointwise mul + inv NTT, BASELINE configs[1]",
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (uniform canonical residues per limb, seeded; rlk broadcast over RCCL)",
            "config": {"workload": workload, "ring_degree": n, "ct_limbs": L, "limb_bits": 60,
                       "plain_modulus": plain, "gadget_base": gbase, "gadget_digits": G,
                       "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"batch-shard x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if dbfv is not None:
            line["config"].update({"dbfv_digits": dbfv[0], "dbfv_base": dbfv[1],
                                   "dbfv_plain_modulus": dbfv[2] or "2^64", "chain_depth": depth})
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
