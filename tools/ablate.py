#!/usr/bin/env python3
"""Experiment harness (not product code): build consensus kernel variants with parts
switched off (-DBCE_ABLATE=mask, -DBCE_SEG32_TM=..., -DBCE_SEG_GRID_PER_CU=...) and time
them on the config-2 workload in ONE process, interleaved rounds (cdna guide §5.4 r24).

  python tools/ablate.py build            # here (hipcc cross-compiles)
  python tools/ablate.py run [--rounds 5] # on the GPU box
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bayesian-consensus-engine_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "ablate_build")

VARIANTS = {
    "pipe": [],
    "pipe_c5": ["-DBCE_PIPE_C32=5"],
    "pipe_ring24": ["-DBCE_PIPE_RING=24"],
    "pipe_l2": ["-DBCE_PIPE_L=2"],
    "lpm": ["-DBCE_FLAT=0"],
    "pipe_noout": ["-DBCE_ABLATE=8"],
    "pipe_nogather": ["-DBCE_ABLATE=2"],
    "pipe_prof": ["-DBCE_PIPE_PROF=1"],
    "pipe_prof_nocheck": ["-DBCE_PIPE_PROF=1", "-DBCE_ABLATE=32"],
    "pipe_nogather_noout": ["-DBCE_ABLATE=10"],
    "pipe_nosort": ["-DBCE_ABLATE=1"],
    "pipe_l2_ngno": ["-DBCE_PIPE_L=2", "-DBCE_ABLATE=10"],
    "pipe_l2_c3": ["-DBCE_PIPE_L=2", "-DBCE_PIPE_C32=3", "-DBCE_PIPE_R32=6"],
    "pipe_c3": ["-DBCE_PIPE_C32=3", "-DBCE_PIPE_R32=6"],
    "pipe_lprio3": ["-DBCE_PIPE_LPRIO=3"],
    "pipe_lprio1": ["-DBCE_PIPE_LPRIO=1"],
    "pipe_nts": ["-DBCE_PIPE_NTS=1"],
    "pipe_nocheck": ["-DBCE_ABLATE=32"],
    "pipe_nts_lprio3": ["-DBCE_PIPE_NTS=1", "-DBCE_PIPE_LPRIO=3"],
}
SRCS = ["capi.hip", "consensus.hip", "elementwise.hip", "tiebreak.hip", "stats.hip", "aggregate.hip"]


def build(names):
    os.makedirs(OUT, exist_ok=True)
    procs = []
    for name in names:
        flags = VARIANTS[name]
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off"] + flags + [os.path.join(CSRC, s) for s in SRCS] + \
              ["-o", os.path.join(OUT, f"lib_{name}.so")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0


def run(names, rounds, steps):
    sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from bench import make_c2

    M, L, S = 1_000_000, 32, 10_000
    off, sid, prob, rel, conf, present = make_c2(M, L, S, 2)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    d = [T(x) for x in (off, sid, prob, rel, conf, present)]
    f64 = dict(dtype=torch.float64, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    outs = [torch.empty(M, **f64), torch.empty(M, **f64), torch.empty(M, **f64), torch.empty(M, **i32),
            torch.empty(M, **i32), torch.empty(M * L, **i32), torch.empty(M * L, **f64), torch.empty(M * L, **f64)]
    from bayesian_engine import batch
    table = batch.SourceTable.from_arrays(d[3], d[4], d[5])
    libs = {}
    for n in names:
        lib = C.CDLL(os.path.join(OUT, f"lib_{n}.so"))
        lib.bce_consensus_csr.restype = C.c_int
        libs[n] = lib
    st = torch.cuda.current_stream()
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731

    def call(lib):
        rc = lib.bce_consensus_csr(p(d[0]), C.c_int64(M), p(d[1]), p(d[2]), C.c_int64(M * L), p(table.relconf),
                                   p(table.bits), C.c_int32(S), C.c_void_p(0), C.c_int64(0), C.c_int32(L), C.c_int32(0),
                                   *[p(o) for o in outs], C.c_void_p(st.cuda_stream))
        assert rc == 0, rc

    res = {n: [] for n in names}
    for n in names:
        for _ in range(3):
            call(libs[n])
    torch.cuda.synchronize()
    for r in range(rounds):
        for n in names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(steps):
                call(libs[n])
            e1.record(st)
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) / steps)
    # reference copy bandwidth (1 GiB read + 1 GiB write)
    a = torch.empty(2**27, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    copy_gbs = 2 * a.numel() * 8 / (e0.elapsed_time(e1) / 10 / 1e3) / 1e9
    summary = {n: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))} for n, v in res.items()}
    summary["_copy_GBps"] = copy_gbs
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["build", "run"])
    ap.add_argument("--only", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    names = a.only.split(",") if a.only else list(VARIANTS)
    if a.what == "build":
        t = time.time()
        build(names)
        print(f"built {len(names)} variants in {time.time() - t:.1f}s")
    else:
        run(names, a.rounds, a.steps)
