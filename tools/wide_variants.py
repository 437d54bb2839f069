#!/usr/bin/env python3
"""Experiment harness (not product code): build variants of libbce_hip.so as source patches
of csrc/ (tools/tab_variants.py's mechanism; the product carries no experiment switches) and
time them on the config-3 workload.

  python tools/wide_variants.py build [names...]     # here (hipcc cross-compiles)
  python tools/wide_variants.py run [names...]       # on the GPU box: one process per variant
                                                     # and mode; JSON lines out

Each line: median ms per planned consensus step (all bins), printed only after the variant's
outputs matched the C restatement (ablations excepted, which are wrong by construction).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import tab_variants  # noqa: E402

OUT = tab_variants.OUT

# Variants of rounds 2-3 (row exchange layout, 6-wave occupancy, no-park, power-of-two bins,
# EXACT np2 split, FAST np2 merge, no DPP fusion, no swap stages, the s_memtime phase timer,
# gather windows, late probabilities, dedup-before-sort, M0 save/restore) were source patches
# of the pre-round-4 kernel; their results are in DESIGN.md §4.2 and profiles/archive/r03*/.  They no
# longer apply to the refactored per-market body and were dropped.
# Round 5: the all-bins team kernel, the rotated sorted-probability layout (kWideSwz) and the
# tie-break's LDS-DMA staging (kTbStageMode 1/2), pre-issued batches (kTbPreBatch) and next-array
# touches (kTbTouchNext) were removed from csrc/ (verdict r04 item 7); their A/Bs are recorded in
# DESIGN.md §4.2 / §4.9 and profiles/archive/r04c, r04e, r04f, r04k, r04m, r04aa.
VARIANTS = {
    "wbase": [],
    # small planned calls without the bin merges / merging below 3 resident rounds (shipped: 6)
    "nomerge": [("consensus.hip", "constexpr double kMergeRounds = 6.0;", "constexpr double kMergeRounds = 0.0;")],
    "merge3": [("consensus.hip", "constexpr double kMergeRounds = 6.0;", "constexpr double kMergeRounds = 3.0;")],
    # C2 tab kernel: the next tile's metadata read after the walk (no spill stores in the tile
    # loop; shipped: at the top of the tile, as round 4)
    "tablate": [("consensus_tab.hip", "constexpr bool kTabMetaEarly = true;", "constexpr bool kTabMetaEarly = false;")],
    # tie-break FULL tiles: staging batches of the predictions / confidences (shipped: 8)
    "tbpc16": [("tiebreak.hip", "constexpr int kTbFullBatchPC = 8;", "constexpr int kTbFullBatchPC = 16;")],
    "tbpc4": [("tiebreak.hip", "constexpr int kTbFullBatchPC = 8;", "constexpr int kTbFullBatchPC = 4;")],
    # tie-break staging / flush without the nontemporal hints (0.727-0.730 vs 0.712 ms, r04j)
    "tbnont": [("tiebreak.hip", "constexpr bool kTbNtLoad = true;", "constexpr bool kTbNtLoad = false;"),
               ("tiebreak.hip", "constexpr bool kTbNtStore = true;", "constexpr bool kTbNtStore = false;")],
    "tbnopre": [("tiebreak.hip", "constexpr bool kTbPrefetchMeta = true;", "constexpr bool kTbPrefetchMeta = false;")],
    # FULL tiles: staging batches (shipped: 8 and 8)
    "tbwr4": [("tiebreak.hip", "constexpr int kTbFullBatchWR = 8;", "constexpr int kTbFullBatchWR = 4;")],
    "tbwr16": [("tiebreak.hip", "constexpr int kTbFullBatchWR = 8;", "constexpr int kTbFullBatchWR = 16;")],
    "tbpc16wr16": [("tiebreak.hip", "constexpr int kTbFullBatchWR = 8;", "constexpr int kTbFullBatchWR = 16;"),
                   ("tiebreak.hip", "constexpr int kTbFullBatchPC = 8;", "constexpr int kTbFullBatchPC = 16;")],
    # C5 MFMA pass: two accumulator chains / no next-batch prefetch (8 waves per SIMD)
    # (shipped: one chain, 8-row batches, the next batch issued before the chain, 6 waves)
    "c5acc2": [("stats.hip", "constexpr bool kMfmaTwoAcc = false;", "constexpr bool kMfmaTwoAcc = true;")],
    "c5nopf": [("stats.hip", "constexpr bool kMfmaPrefetch = true;", "constexpr bool kMfmaPrefetch = false;")],
    # EXACT piped chain wave with the 8-term chain_add (shipped: chain_add_deep, 16-term steps)
    "nodeep": [("consensus_wide.hip", "constexpr bool kWideChainDeep = true;", "constexpr bool kWideChainDeep = false;")],
    # EXACT chains on every lane of the chain wave (lane % 3 picks the chain; shipped: lanes 0..2)
    "chain64": [("consensus_wide.hip", "constexpr bool kWideChain3 = true;", "constexpr bool kWideChain3 = false;")],
    # C5 exact pass 1 on 256- / 512-thread workgroups (shipped: 1024)
    "c5b256": [("stats.hip", "constexpr int kVoteBlock = 1024;", "constexpr int kVoteBlock = 256;")],
    "c5b512": [("stats.hip", "constexpr int kVoteBlock = 1024;", "constexpr int kVoteBlock = 512;")],
    # C5 exact pass 1: blocks in launch order over the columns (shipped: one contiguous column
    # slice per XCD)
    "c5noxcd": [("stats.hip", "constexpr bool kVoteXcd = true;", "constexpr bool kVoteXcd = false;")],
    # C5 exact and MFMA passes in launch order (shipped: one contiguous column slice per XCD)
    "c5noxcd": [("stats.hip", "constexpr bool kVoteXcd = true;", "constexpr bool kVoteXcd = false;")],
    "wdiv": [("consensus_wide.hip", "constexpr bool kWideFastRecip = true;", "constexpr bool kWideFastRecip = false;")],
    # namespace pass without its nontemporal hints (0.1752 vs 0.1665 ms, r04t)
    "nsnont": [("elementwise.hip", "constexpr bool kNsNtLoad = true;", "constexpr bool kNsNtLoad = false;"),
               ("elementwise.hip", "constexpr bool kNsNtStore = true;", "constexpr bool kNsNtStore = false;")],
    # f4: the last chunk's chains in the compiler's 8-term loop inside the chunk loop (shipped:
    # after the loop, asm, four 4-term batches in flight)
    "aggnoasm": [("aggregate.hip", "constexpr bool kAggChainAsm = true;", "constexpr bool kAggChainAsm = false;")],
    "aggw1": [("aggregate.hip", "constexpr int kAggWpe = 6;", "constexpr int kAggWpe = 1;")],
    "tab4w": [("consensus_tab.hip", "constexpr int kTabWaves = 8;", "constexpr int kTabWaves = 4;")],
    "tbkvsort": [("tiebreak.hip", "constexpr bool kTbFullKeysInLds = true;", "constexpr bool kTbFullKeysInLds = false;")],
    # tie-break without the FULL-tile kernel (one general launch)
    "tbnofull": [("tiebreak.hip", "bool split = !EXOTIC && a.rmode == 0 && al16(a.pred)",
                  "const bool split = false && al16(a.pred)")],
    # ---- ablations (timing only; outputs are wrong by construction -- no parity gate) ----
    # the sort network run twice (the second pass on sorted keys costs the same)
    "xsort2": [("consensus_wide.hip", "  wide_sort<NN, NW, R>(key, sX, t, lane);\n",
                "  wide_sort<NN, NW, R>(key, sX, t, lane);\n  wide_sort<NN, NW, R>(key, sX, t, lane);\n")],
    # no relconf / present-bit gathers (constant rows)
    "xnogather": [("consensus_wide.hip", "rc[i] = a.relconf[sids[i]];", "rc[i] = make_double2(0.5 + 1e-9 * sids[i], 0.25);"),
                  ("consensus_wide.hip", "pwd[i] = a.pbits[sids[i] >> 5];", "pwd[i] = 0xFFFFFFFFu;")],
    # no normalizedWeight phase
    "xnonw": [("consensus_wide.hip", "  if (a.nweight) {  // core.py:151", "  if (false) {  // core.py:151")],
}
ABLATIONS = {"xsort2", "xnogather", "xnonw"}


def build(names):
    tab_variants.build(names, VARIANTS)


def one(name, mode, reps):
    sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from bayesian_engine import _native as N, batch
    from bench_extra import make_c3

    M, off, sid, prob, (rel, conf, present), _ = make_c3()
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(present))
    d = [T(off), T(sid), T(prob)]
    plan = batch.Plan.build(off, d[0].device)
    res = batch._alloc(M, int(off[-1]), d[0].device, True, True)
    t0 = time.time()
    while time.time() - t0 < 1.0:  # clock ramp
        batch.consensus(*d, table, plan=plan, mode=mode, out=res)
        torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        batch.consensus(*d, table, plan=plan, mode=mode, out=res)
        e1.record(st)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    N.check_faults()
    # parity gate: every output of the timed variant against the C restatement (bit for bit;
    # FAST floats within 1e-9) -- a wrong variant prints no time (round 3 once timed a variant
    # that skipped part of the per-unique loop)
    if name not in ABLATIONS:
        from bench import cpu_consensus_threaded, host_threads
        from bench_extra import _parity_c3
        cpu = cpu_consensus_threaded(off, sid, prob, rel, conf, present, host_threads())
        ok, dev = _parity_c3(res, cpu, off, exact=(mode == "exact"))
        if not all(ok.values()):
            print(json.dumps({"variant": name, "mode": mode, "parity": False, "outputs": ok, "max_dev": dev}),
                  flush=True)
            raise SystemExit(3)
    out = {"variant": name, "mode": mode, "parity": name not in ABLATIONS or "n/a (ablation)",
           "median_ms": ms[len(ms) // 2], "min_ms": ms[0]}
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
        names = [n for n in names if os.path.exists(os.path.join(OUT, n, "libbce_hip.so"))]
        for n in names:
            for mode in args.modes.split(","):
                env = dict(os.environ, BCE_LIB=os.path.join(OUT, n, "libbce_hip.so"))
                t0 = time.time()
                rc = subprocess.run([sys.executable, __file__, "one", n, "--modes", mode, "--reps", str(args.reps)],
                                    env=env, timeout=300).returncode
                if rc != 0:
                    raise SystemExit(f"variant {n} ({mode}) failed rc={rc}")
                print(f"# {n} {mode} {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
