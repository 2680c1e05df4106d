#!/usr/bin/env python3
"""Standalone NTT benchmark (BASELINE configs[1]): n=4096, 60-bit q, batch of polys resident in HBM.

Times forward NTT, pointwise mul and inverse NTT separately with HIP events on the library's
stream and prints algorithmic GB/s (16*n bytes per polynomial per transform, 24*n per pointwise
mul).  Used under rocprofv3 (--kernel-trace / --pmc) to attribute time and HBM bytes.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from exacto_amd._ffi import HipContext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--q", type=int, default=1152921504606830593)
ap.add_argument("--polys", type=int, default=16384)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()

dev = torch.device("cuda", 0)
ctx = HipContext(args.n, [args.q], plain_modulus=65537)
s = torch.cuda.current_stream()
ctx.set_stream(s.cuda_stream)
g = torch.Generator(device=dev)
g.manual_seed(2)
a = torch.randint(0, args.q, (args.polys, args.n), generator=g, dtype=torch.int64, device=dev)
b = torch.randint(0, args.q, (args.polys, args.n), generator=g, dtype=torch.int64, device=dev)
torch.cuda.synchronize()


def timed(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.reps


P, n = args.polys, args.n
t_f = timed(lambda: ctx.rns_fwd_dev(a, P))
t_i = timed(lambda: ctx.rns_inv_dev(a, P))
t_m = timed(lambda: ctx.rns_mul_dev(a, b, a, P))
gb = lambda bytes_, ms: bytes_ / (ms * 1e-3) / 1e9
print(json.dumps({
    "polys": P, "n": n,
    "fwd_ms": round(t_f, 4), "fwd_GBs": round(gb(16 * n * P, t_f), 1),
    "fwd_polys_per_us": round(P / (t_f * 1e3), 2),
    "inv_ms": round(t_i, 4), "inv_GBs": round(gb(16 * n * P, t_i), 1),
    "mul_ms": round(t_m, 4), "mul_GBs": round(gb(24 * n * P, t_m), 1),
}))
