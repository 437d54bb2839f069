#!/usr/bin/env python3
"""Experiment harness (not product code): build variants of libbce_hip.so with compile-time
switches of the wide-market kernel (consensus_wide.hip) and time them on the config-3 workload.

  python tools/wide_variants.py build [names...]     # here (hipcc cross-compiles)
  python tools/wide_variants.py run [names...]       # on the GPU box: one process per variant
                                                     # and mode; JSON lines out

Each line: median ms per planned consensus step (all bins) and, for *prof* variants, the
per-phase cycle split of the wide kernels' waves (s_memtime deltas summed over waves,
per market of the wide bins).
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
    "base": [],
    "prof": ["-DBCE_WIDE_PROF=1"],
    "hr3": ["-DBCE_WIDE_HR=3"],
    "hr4": ["-DBCE_WIDE_HR=4"],
    "kwr32": ["-DBCE_WIDE_KWR=32"],
    "kwr96": ["-DBCE_WIDE_KWR=96"],
    "nopipe": ["-DBCE_WIDE_PIPE=0"],
    "w2": ["-DBCE_WIDE_WPE_BIG=2"],
    "wpe4": ["-DBCE_WIDE_WPE=4"],  # 4 waves/SIMD (<= 128 VGPRs) for the 1- and 2-wave kernels too
    "wpe3": ["-DBCE_WIDE_WPE=3"],
    "nwb0": ["-DBCE_WIDE_NWB=0"],
    "nwbf1": ["-DBCE_WIDE_NWBF=1"],
    "nwbf2": ["-DBCE_WIDE_NWBF=2"],
}
PHASES = ["keys+next sids", "sort", "probs+leaders", "run sums+products+stores", "stage barrier", "chain", "tail",
          "gather wait"]


def build(names):
    for name in names:
        d = os.path.join(OUT, "wide_" + name)
        os.makedirs(d, exist_ok=True)
        procs, objs = [], []
        for src in SRCS:
            o = os.path.join(d, src.replace(".hip", ".o"))
            objs.append(o)
            cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                   "-fno-fast-math", "-munsafe-fp-atomics", "-w", *VARIANTS[name], "-c", os.path.join(CSRC, src),
                   "-o", o]
            procs.append(subprocess.Popen(cmd))
        for p in procs:
            if p.wait() != 0:
                raise SystemExit(f"build of {name} failed")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libbce_hip.so"), *objs], check=True)
        print("built", name, flush=True)


def one(name, mode, reps):
    sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from bayesian_engine import _native as N, batch
    from bench_extra import make_c3

    M, off, sid, prob, (rel, conf, present) = make_c3()
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(present))
    d = [T(off), T(sid), T(prob)]
    plan = batch.Plan.build(off, d[0].device)
    res = batch._alloc(M, int(off[-1]), d[0].device, True, True)
    t0 = time.time()
    while time.time() - t0 < 1.0:  # clock ramp
        batch.consensus(*d, table, plan=plan, mode=mode, out=res)
        torch.cuda.synchronize()
    lib = N.lib()
    prof = hasattr(lib, "bce_wide_prof_read")
    buf = (C.c_ulonglong * 8)()
    if prof:
        lib.bce_wide_prof_read(buf)
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        batch.consensus(*d, table, plan=plan, mode=mode, out=res)
        e1.record(st)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    out = {"variant": name, "mode": mode, "median_ms": ms[len(ms) // 2], "min_ms": ms[0]}
    if prof:
        lib.bce_wide_prof_read(buf)
        v = list(buf)[:8]
        lens = np.diff(off)
        wide = int(((lens > 64) & (lens <= 4096)).sum())
        tot = sum(v)
        out["phases_wave_cyc_per_market"] = {k: round(x / reps / wide) for k, x in zip(PHASES, v)}
        out["phases_pct"] = {k: round(100 * x / max(tot, 1), 1) for k, x in zip(PHASES, v)}
    N.check_faults()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run", "one"])
    ap.add_argument("names", nargs="*")
    ap.add_argument("--modes", default="exact,fast")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    names = args.names or list(VARIANTS)
    if args.cmd == "build":
        build(names)
    elif args.cmd == "one":
        one(names[0], args.modes, args.reps)
    else:
        names = [n for n in names if os.path.exists(os.path.join(OUT, "wide_" + n, "libbce_hip.so"))]
        for n in names:
            for mode in args.modes.split(","):
                env = dict(os.environ, BCE_LIB=os.path.join(OUT, "wide_" + n, "libbce_hip.so"))
                t0 = time.time()
                rc = subprocess.run([sys.executable, __file__, "one", n, "--modes", mode, "--reps", str(args.reps)],
                                    env=env, timeout=300).returncode
                if rc != 0:
                    raise SystemExit(f"variant {n} ({mode}) failed rc={rc}")
                print(f"# {n} {mode} {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
