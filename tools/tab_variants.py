#!/usr/bin/env python3
"""Experiment harness (not product code): build variants of libbce_hip.so with compile-time
switches of the LDS-table kernel (consensus_tab.hip) and time them on the config-2 workload.

  python tools/tab_variants.py build [names...]     # here (hipcc cross-compiles)
  python tools/tab_variants.py run [--rounds 3]      # on the GPU box: one process per variant
                                                     # and round, interleaved; JSON lines out

A variant named *prof* is built with -DBCE_TAB_PROF=1 and also reports the per-phase cycle
split of the kernel's waves (s_memtime deltas summed over waves, per tile).
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
SRCS = ["capi.hip", "consensus.hip", "consensus_tab.hip", "consensus_wide.hip", "elementwise.hip", "tiebreak.hip",
        "stats.hip", "aggregate.hip"]

VARIANTS = {
    "base": [],  # the product defaults (8 waves, BCE_TAB_NT=3, BCE_EW_NT=2)
    "w4": ["-DBCE_TAB_WAVES=4"],
    "w8": ["-DBCE_TAB_WAVES=8"],
    "w4_prof": ["-DBCE_TAB_WAVES=4", "-DBCE_TAB_PROF=1"],
    "w8_prof": ["-DBCE_TAB_WAVES=8", "-DBCE_TAB_PROF=1"],
    "p64": ["-DBCE_TAB_PIECE=64"],
    "p64_prof": ["-DBCE_TAB_PIECE=64", "-DBCE_TAB_PROF=1"],
    "nt1": ["-DBCE_TAB_NT=1"],  # nontemporal signal loads
    "nt2": ["-DBCE_TAB_NT=2"],  # nontemporal per-unique stores
    "nt3": ["-DBCE_TAB_NT=3"],
    "nt7": ["-DBCE_TAB_NT=7"],
    "nt3_w8": ["-DBCE_TAB_NT=3", "-DBCE_TAB_WAVES=8"],
    "nt3_p64": ["-DBCE_TAB_NT=3", "-DBCE_TAB_PIECE=64"],
    "nt3_prof": ["-DBCE_TAB_NT=3", "-DBCE_TAB_PROF=1"],
    "base_prof": ["-DBCE_TAB_PROF=1"],
    "map0": ["-DBCE_TAB_MAP=0"],
    "prio0": ["-DBCE_TAB_PRIO=0"],
    "plx": ["-DBCE_TAB_PLX=1"],
    "xord_old": ["-DBCE_TAB_XORD_OLD=1"],
    "ewg16": ["-DBCE_EW_GRID_CAP=16"],
    "agg8": ["-DBCE_AGG_CAP=8"],  # f4: 8 workgroups per CU looping over groups (bench --config agg)  # elementwise kernels: 16 workgroups per CU (bench --config c4 / ns)
    "ew1": ["-DBCE_EW_NT=1"],  # config-4 replay_step variants (bench.py --config c4)
    "ew2": ["-DBCE_EW_NT=2"],
    "ew3": ["-DBCE_EW_NT=3"],
    "ew6": ["-DBCE_EW_NT=6"],
    "nt7_w8": ["-DBCE_TAB_NT=7", "-DBCE_TAB_WAVES=8"],
    "nt3_w8_r4": ["-DBCE_TAB_NT=3", "-DBCE_TAB_WAVES=8", "-DBCE_TAB_RING=4"],
    "nt3_w8_r6": ["-DBCE_TAB_NT=3", "-DBCE_TAB_WAVES=8", "-DBCE_TAB_RING=6"],
    "wide_nt": ["-DBCE_WIDE_AUX=2"],  # config-3 wide kernel: nontemporal sid/prob buffer loads
}
PHASES = ["load+xpose", "valid+sort", "walk", "per_market", "compaction", "per_unique_stores"]


def build(names):
    procs = []
    for name in names:
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        objs = []
        for src in SRCS:
            o = os.path.join(d, src.replace(".hip", ".o"))
            objs.append(o)
            cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                   "-fno-fast-math", "-munsafe-fp-atomics", "-w", *VARIANTS[name], "-c", os.path.join(CSRC, src),
                   "-o", o]
            procs.append((name, subprocess.Popen(cmd)))
        for _, p in procs:
            if p.wait() != 0:
                raise SystemExit(f"build of {name} failed")
        procs = []
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libbce_hip.so"), *objs], check=True)
        print("built", name, flush=True)


def one(name, reps):
    sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from bayesian_engine import _native as N, batch
    from bench import make_c2

    M, L, S = 1_000_000, 32, 10_000
    off, sid, prob, rel, conf, present = make_c2(M, L, S, 2)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(present))
    d = [T(off), T(sid), T(prob)]
    res = batch._alloc(M, M * L, d[0].device, True, True)
    for _ in range(300):  # clock ramp
        batch.consensus(*d, table, max_len=L, out=res)
    torch.cuda.synchronize()
    lib = N.lib()
    prof = hasattr(lib, "bce_tab_prof_read")
    buf = (C.c_ulonglong * 8)()
    if prof:
        lib.bce_tab_prof_read(buf)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        batch.consensus(*d, table, max_len=L, out=res)
        e1.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    out = {"variant": name, "median_ms": ms[len(ms) // 2], "min_ms": ms[0]}
    if prof:
        lib.bce_tab_prof_read(buf)
        v = list(buf)[:6]
        tiles = (M + 63) // 64
        tot = sum(v)
        out["phases_cyc_per_tile"] = {k: round(x / reps / tiles) for k, x in zip(PHASES, v)}
        out["phases_pct"] = {k: round(100 * x / max(tot, 1), 1) for k, x in zip(PHASES, v)}
    if os.environ.get("TAB_NOCHECK") is None:
        N.check_faults()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run", "one"])
    ap.add_argument("names", nargs="*")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=100)
    args = ap.parse_args()
    names = args.names or list(VARIANTS)
    if args.cmd == "build":
        build(names)
    elif args.cmd == "one":
        one(names[0], args.reps)
    else:
        names = [n for n in names if os.path.exists(os.path.join(OUT, n, "libbce_hip.so"))]
        for r in range(args.rounds):
            for n in names:
                env = dict(os.environ, BCE_LIB=os.path.join(OUT, n, "libbce_hip.so"))
                t0 = time.time()
                rc = subprocess.run([sys.executable, __file__, "one", n, "--reps", str(args.reps)], env=env,
                                    timeout=300).returncode
                if rc != 0:
                    raise SystemExit(f"variant {n} failed rc={rc}")
                print(f"# round {r} {n} {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
