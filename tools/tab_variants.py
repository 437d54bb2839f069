#!/usr/bin/env python3
"""Experiment harness (not product code): build variants of libbce_hip.so as SOURCE PATCHES of
csrc/ (the product source carries no experiment switches) and time them on the config-2
workload.  Every timed variant is checked against the C restatement (all eight outputs, bit
for bit) before its time is printed: a variant that computes something else prints
{"parity": false} and no time, and the run stops.

  python tools/tab_variants.py build [names...]     # here (hipcc cross-compiles)
  python tools/tab_variants.py run [--rounds 3]      # on the GPU box: one process per variant
                                                     # and round, interleaved; JSON lines out

A variant is a list of (file, old text, new text) replacements applied to a copy of csrc/;
a replacement whose old text is missing fails the build (the patch went stale).
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bayesian-consensus-engine_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "bin", "variants")  # gitignored; travels to the GPU box
SRCS = ["capi.hip", "consensus.hip", "consensus_tab.hip", "consensus_wide.hip", "elementwise.hip", "tiebreak.hip",
        "stats.hip", "aggregate.hip"]
CPP_SRCS = ["jsonl.cpp"]

_XPOSE_NEW = """  for (int i = 0; i < N; ++i)
    if (!(i & 4)) bfly_r8(r[i], r[i | 4], lane);
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (!(i & 8)) bfly_pl16(r[i], r[i | 8]);
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (!(i & 16)) bfly_pl32(r[i], r[i | 16]);
}"""
_XPOSE_OLD = """  for (int i = 0; i < N; ++i)
    if (!(i & 16)) bfly_pl32(r[i], r[i | 16]);
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (!(i & 8)) bfly_pl16(r[i], r[i | 8]);
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (!(i & 4)) bfly_r8(r[i], r[i | 4], lane);
}"""

VARIANTS = {
    "base": [],  # the product source as is
    # round-2 order of the transposes (row_ror:8 first): fewer spills, measured slower
    "xord_r8first": [("consensus_tab.hip", _XPOSE_OLD, _XPOSE_NEW)],
    "w4": [("consensus_tab.hip", "constexpr int kTabWaves = 8;", "constexpr int kTabWaves = 4;")],
    "prio0": [("consensus_tab.hip", "__builtin_amdgcn_s_setprio(", "(void)(")],
}


def _patched_src(name, variants=None):
    variants = VARIANTS if variants is None else variants
    # pkg/csrc + include side by side, as in the repo (csrc includes ../../include/bce.h)
    top = os.path.join(OUT, name, "tree")
    if os.path.isdir(top):
        shutil.rmtree(top)
    d = os.path.join(top, "pkg", "csrc")
    shutil.copytree(CSRC, d)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    for fn, old, new in variants[name]:
        path = os.path.join(d, fn)
        text = open(path).read()
        if old not in text:
            raise SystemExit(f"variant {name}: patch for {fn} does not apply (stale)")
        with open(path, "w") as f:
            f.write(text.replace(old, new))
    return d


def build(names, variants=None):
    procs = []
    for name in names:
        d = os.path.join(OUT, name)
        src = _patched_src(name, variants)
        objs = []
        for fn in SRCS:
            o = os.path.join(d, fn.replace(".hip", ".o"))
            objs.append(o)
            cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                   "-fno-fast-math", "-munsafe-fp-atomics", "-w", "-I", src, "-c", os.path.join(src, fn), "-o", o]
            procs.append((name, subprocess.Popen(cmd)))
        for _, p in procs:
            if p.wait() != 0:
                raise SystemExit(f"build of {name} failed")
        procs = []
        for fn in CPP_SRCS:  # host-only C++ (the JSONL front end)
            o = os.path.join(d, fn.replace(".cpp", ".o"))
            objs.append(o)
            subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-pthread", "-D__HIP_PLATFORM_AMD__",
                            "-I/opt/rocm/include", "-w", "-I", src, "-c", os.path.join(src, fn), "-o", o], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o",
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
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        batch.consensus(*d, table, max_len=L, out=res)
        e1.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    if os.environ.get("TAB_NOCHECK") is None:
        N.check_faults()
    # parity gate: a variant whose outputs differ from the restatement prints no time
    from bench import cpu_consensus_threaded, host_threads, parity_all_outputs
    cpu = cpu_consensus_threaded(off, sid, prob, rel, conf, present, host_threads())
    ok = parity_all_outputs(res, cpu, off, True)
    if not all(ok.values()):
        print(json.dumps({"variant": name, "parity": False, "outputs": ok}), flush=True)
        raise SystemExit(3)
    out = {"variant": name, "parity": True, "median_ms": ms[len(ms) // 2], "min_ms": ms[0]}
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
