#!/usr/bin/env python3
"""Config-3 speed-of-light probes (GPU box, repo root; tools/sol_c3.hip, built on the CPU into
tools/bin/libsol_c3.so): the real C3 batch, its real unique lists (from one FAST consensus step
of the product), and probes that move the same bytes with trivial compute -- flat grid-stride
streams, and one workgroup per market at the wide kernel's occupancy and at higher ones.  Prints
one JSON object: each probe's time per step, the product's own step, and the algorithmic bytes.

  python3 tools/sol_c3.py [--sources 1000000] [--reps 20]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))

FIELDS = ["offsets", "sid", "prob", "order", "n_markets", "uoff", "ulist", "n_uniques", "relconf", "bits",
          "usid", "weight", "nweight", "cons", "conf", "tw", "nu", "err", "sink"]


class SolArgs(C.Structure):
    _fields_ = [(f, C.c_int64 if f in ("n_markets", "n_uniques") else C.c_void_p) for f in FIELDS]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sources", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from bench_extra import make_c3
    from bayesian_engine import batch

    M, off, sid, prob, (rel, conf, pres), _ = make_c3(1, 0, S=a.sources)
    dev = torch.device("cuda", 0)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(pres))
    d_off, d_sid, d_prob = T(off), T(sid), T(prob)
    plan = batch.Plan.build(off, dev)
    N = int(off[-1])
    res = batch._alloc(M, N, dev, True, True)
    st = torch.cuda.current_stream(dev)

    def product():
        batch.consensus(d_off, d_sid, d_prob, table, plan=plan, mode="fast", out=res)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    t_product = timeit(product)
    nu = res.n_unique.to(torch.int64)
    uoff = torch.zeros(M + 1, dtype=torch.int64, device=dev)
    uoff[1:] = torch.cumsum(nu, 0)
    U = int(uoff[-1].item())
    umk = torch.repeat_interleave(torch.arange(M, device=dev, dtype=torch.int32), nu)
    pos = d_off[:-1].repeat_interleave(nu) + (torch.arange(U, device=dev) - uoff[:-1].repeat_interleave(nu))
    ulist = (res.usid[pos] & 0x7FFFFFFF).to(torch.int32).contiguous()
    out = {k: torch.empty_like(v) for k, v in (("usid", res.usid), ("weight", res.weight), ("nweight", res.nweight))}
    mo = {k: torch.empty(M, dtype=torch.float64, device=dev) for k in ("cons", "conf", "tw")}
    mi = {k: torch.empty(M, dtype=torch.int32, device=dev) for k in ("nu", "err")}
    sink = torch.zeros(8, dtype=torch.float64, device=dev)
    keep = [d_off, d_sid, d_prob, plan.order, uoff, ulist, table.relconf, table.bits, sink, umk]
    args = SolArgs(offsets=d_off.data_ptr(), sid=d_sid.data_ptr(), prob=d_prob.data_ptr(), order=plan.order.data_ptr(),
                   n_markets=M, uoff=uoff.data_ptr(), ulist=ulist.data_ptr(), n_uniques=U,
                   relconf=table.relconf.data_ptr(), bits=table.bits.data_ptr(), usid=out["usid"].data_ptr(),
                   weight=out["weight"].data_ptr(), nweight=out["nweight"].data_ptr(), cons=mo["cons"].data_ptr(),
                   conf=mo["conf"].data_ptr(), tw=mo["tw"].data_ptr(), nu=mi["nu"].data_ptr(),
                   err=mi["err"].data_ptr(), sink=sink.data_ptr())
    lib = C.CDLL(os.path.join(ROOT, "tools", "bin", "libsol_c3.so"))
    lib.sol_c3_run.argtypes = [C.POINTER(SolArgs), C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    touched = int(torch.unique(d_sid).numel())
    alg = 12 * N + 8 * (M + 1) + 32 * M + 20 * U + 17 * touched
    res_out = {"sources": a.sources, "markets": M, "signals": N, "uniques": U, "algorithmic_bytes": alg,
               "probe_extra_bytes": 4 * U, "product_fast_ms": t_product,
               "product_frac": alg / (t_product * 1e-3) / 8e12, "probes": {}}
    names = {0: "flat (signals, uniques, markets: three grid-stride kernels)",
             1: "market, 512 threads, 2 per CU (the <8,8> wide kernel's shape)",
             2: "market, 256 threads, 4 per CU", 3: "market, 256 threads, 8 per CU (8 waves per SIMD)",
             4: "market, 64 threads, 32 per CU (8 waves per SIMD)"}
    for v, nm in names.items():
        fn = lambda v=v: lib.sol_c3_run(C.byref(args), C.c_void_p(umk.data_ptr()), v, N & 0xFFFFFFFF, N >> 32,  # noqa: E731
                                        C.c_void_p(st.cuda_stream))
        ms = timeit(fn)
        res_out["probes"][nm] = {"ms": ms, "frac_of_algorithmic": alg / (ms * 1e-3) / 8e12,
                                 "GBps_moved": (alg + 4 * U) / (ms * 1e-3) / 1e9}
        print(f"[sol_c3] {nm}: {ms:.4f} ms", file=sys.stderr, flush=True)
    del keep
    print(json.dumps(res_out))


if __name__ == "__main__":
    main()
