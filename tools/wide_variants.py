#!/usr/bin/env python3
"""Experiment harness (not product code): build variants of libbce_hip.so as source patches
of csrc/ (tools/tab_variants.py's mechanism; the product carries no experiment switches) and
time them on the config-3 workload.

  python tools/wide_variants.py build [names...]     # here (hipcc cross-compiles)
  python tools/wide_variants.py run [names...]       # on the GPU box: one process per variant
                                                     # and mode; JSON lines out

Each line: median ms per planned consensus step (all bins).
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

VARIANTS = {
    "wbase": [],
    # round-2 thread-major exchange rows (2-way bank conflicts) instead of 4-key planes
    "wrows": [("consensus_wide.hip", "buf + (r >> 2) * PL + t * 4)", "buf + t * R + r)"),
              ("consensus_wide.hip", "buf + (r >> 2) * PL + (t ^ MT) * 4)", "buf + (t ^ MT) * R + r)")],
    # the 6-wave kernel at 5 waves per SIMD (three workgroups per CU, spills) instead of 4
    "w6wpe5": [("consensus_wide.hip", "static constexpr int WPE = kWideWPE;",
                "static constexpr int WPE = (NW == 6) ? 5 : kWideWPE;")],
    # tie-break lane-per-market kernel at the compiler's choice (1 wave per SIMD, no spills)
    "tbocc1": [("tiebreak.hip", "__attribute__((amdgpu_waves_per_eu(2, 2))) ", "")],
    # FAST nweight from the weight output read-back instead of the LDS park (round 2)
    "wnopark": [("consensus_wide.hip", "const bool park = FAST && wback && u <= WFREE;", "const bool park = false;")],
    # power-of-two bins only: 1025..2048 on 4 waves, 2049..4096 on 8 (round 2)
    "wpow2": [("consensus_wide.hip", "  if (max_len <= 1536) return launch_wide<3, 8, FAST, 4>(a, st);\n", ""),
              ("consensus_wide.hip", "  if (max_len <= 3072) return launch_wide<6, 8, FAST, 8>(a, st);\n", "")],
    # EXACT: the non-power-of-two bins in launches of their own (as FAST) instead of riding
    # with the power-of-two bin above them
    "wsplitx": [("consensus.hip", "const bool merge_np2 = mode == BCE_MODE_EXACT;", "const bool merge_np2 = false;")],
    # FAST too: the non-power-of-two bins ride with the bin above them (power-of-two kernels)
    "wmergef": [("consensus.hip", "const bool merge_np2 = mode == BCE_MODE_EXACT;", "const bool merge_np2 = true;")],
    # round-2/3 lane stages: v_mov_b32_dpp + v_cmp + s_xor + v_cndmask per key (no DPP fusion)
    "wnodpp": [("consensus_wide.hip", "if constexpr (R == 8 && dpp_fusable(MK)) {", "if constexpr (false) {")],
    # half-cleaners across lane bits 4/5 through permlane + compare in VCC instead of the swap trick
    "wnoswap": [("consensus_wide.hip", "if constexpr (!flip && (MK == 16 || MK == 32)) {", "if constexpr (false) {")],
    # phase timer (s_memtime stamps of wave 0 per market, summed per workgroup size): timing aid only
    "wprof": [("consensus_wide.hip", "namespace bce {\nnamespace {\n\nconstexpr int ilog2c",
               "__device__ unsigned long long g_wprof[16 * 8];\n#define WPS(p) { const unsigned long long _n = __builtin_amdgcn_s_memtime(); pacc[p] += _n - pt0; pt0 = _n; }\n"
               "namespace bce {\nnamespace {\n\nconstexpr int ilog2c"),
              ("consensus_wide.hip", "  for (int64_t li = blockIdx.x; li < a.n_list; li += G) {\n",
               "  unsigned long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n  unsigned long long pt0 = 0;\n"
               "  for (int64_t li = blockIdx.x; li < a.n_list; li += G) {\n    pt0 = __builtin_amdgcn_s_memtime();\n"),
              ("consensus_wide.hip", "    // ---- 2. sort (core.py:103", "    WPS(0);\n    // ---- 2. sort (core.py:103"),
              ("consensus_wide.hip", "    wide_sort<NN, NW, R>(key, sX, t, lane);\n", "    wide_sort<NN, NW, R>(key, sX, t, lane);\n    WPS(1);\n"),
              ("consensus_wide.hip", "    __syncthreads();  // (a) input-order", "    __syncthreads(); WPS(2); // (a) input-order"),
              ("consensus_wide.hip", "    __syncthreads();  // (b) every read", "    __syncthreads(); WPS(3); // (b) every read"),
              ("consensus_wide.hip", "    __syncthreads();  // (c) sorted probs", "    __syncthreads(); WPS(4); // (c) sorted probs"),
              ("consensus_wide.hip", "    // ---- 5. next market's probabilities", "    WPS(5);\n    // ---- 5. next market's probabilities"),
              ("consensus_wide.hip", "    __syncthreads();  // totals + w[j] visible", "    __syncthreads(); WPS(6); // totals + w[j] visible"),
              ("consensus_wide.hip", """          }
        }
      }
    }
  }
}

template <int NW, int R, bool FAST, int NN = NW>""", """          }
        }
      }
    }
    WPS(7);
  }
  if (t == 0)
    for (int p = 0; p < 8; ++p) atomicAdd(&g_wprof[NW * 8 + p], pacc[p]);
}

template <int NW, int R, bool FAST, int NN = NW>"""),
              ("consensus_wide.hip", "}  // namespace bce\n", """}  // namespace bce

extern "C" int bce_debug_wprof(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wprof), sizeof(g_wprof)) != hipSuccess) return 1;
  static unsigned long long zero[16 * 8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_wprof), zero, sizeof(g_wprof)) != hipSuccess;
}
""")],
    # more waves per SIMD for the 3-wave and 1-wave kernels (register budget 102 / 85)
    "w3wpe5": [("consensus_wide.hip", "static constexpr int WPE = kWideWPE;",
                "static constexpr int WPE = (NW == 3) ? 5 : kWideWPE;")],
    "w1wpe5": [("consensus_wide.hip", "static constexpr int WPE = kWideWPE;",
                "static constexpr int WPE = (NW == 1) ? 5 : kWideWPE;")],
    "w1wpe6": [("consensus_wide.hip", "static constexpr int WPE = kWideWPE;",
                "static constexpr int WPE = (NW == 1) ? 6 : kWideWPE;")],
    "w36wpe5": [("consensus_wide.hip", "static constexpr int WPE = kWideWPE;",
                "static constexpr int WPE = (NW == 3 || NW == 6) ? 5 : kWideWPE;")],
    # two rounds of uniques with their gathers in flight together (round 2/3 default; +6%)
    "whr2": [("consensus_wide.hip", "constexpr int kWideHR = 1;", "constexpr int kWideHR = 2;")],
    # (each market's probabilities loaded at its start and staged after the sort instead of one
    # market ahead: +2.6% fast, -0.6% exact, profiles/r03k/wide_probs_late_ab.txt)
    # (alternating the wide bins of a market shard between st and the side stream -- bins under
    # 4 rounds of resident workgroups -- made the 1/8 shard step slower, 0.241 -> 0.277 ms,
    # profiles/r03k/c3_shards_alt.json; not kept)
    # two rounds of gathers in flight for the 1-wave kernels only (lower register pressure): no gain
    "whr2nw1": [("consensus_wide.hip", "static constexpr int HR = (R < kWideHR) ? R : kWideHR;",
                 "static constexpr int HR = (NW == 1) ? ((R < 2) ? R : 2) : kWideHR;")],
    # the K = 32R flip stage through the generic lane exchange (compare in VCC)
    "wnoflip31": [("consensus_wide.hip", "if constexpr (flip && MK == 31) {", "if constexpr (false) {")],
    # wave-crossing stages with the per-key compare/select of round 2 instead of a uniform min/max
    "wxwsel": [("consensus_wide.hip", """    if (__builtin_amdgcn_readfirstlane((int)lower)) {
#pragma unroll
      for (int r = 0; r < R; ++r) key[r] = min(key[r], y[flip ? R - 1 - r : r]);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) key[r] = max(key[r], y[flip ? R - 1 - r : r]);
    }""", """#pragma unroll
    for (int r = 0; r < R; ++r) {
      const unsigned yr = y[flip ? R - 1 - r : r];
      key[r] = ((key[r] < yr) == lower) ? key[r] : yr;
    }""")],
    # per-unique stores without the nontemporal hint (FAST +0.5..1%)
    "wtst": [("consensus_wide.hip", """            __builtin_nontemporal_store((int32_t)sids[i] | (((pwd[i] >> (sids[i] & 31)) & 1u) ? 0 : (int32_t)0x80000000), &a.usid[p]);
          if (a.weight) __builtin_nontemporal_store(vw[i], &a.weight[p]);""", """            a.usid[p] = (int32_t)sids[i] | (((pwd[i] >> (sids[i] & 31)) & 1u) ? 0 : (int32_t)0x80000000);
          if (a.weight) a.weight[p] = vw[i];"""),
             ("consensus_wide.hip", "            if (jj < u) __builtin_nontemporal_store((tw > 0.0) ? wj[k] / tw : 0.0, &a.nweight[off + jj]);",
              "            if (jj < u) a.nweight[off + jj] = (tw > 0.0) ? wj[k] / tw : 0.0;")],
    # (a window of 1-3 rounds of gathers issued ahead of the round that uses them measured
    # slower than one round at a time: 1.373-1.493 vs 1.346 ms, profiles/r03w/ab.txt)
    # lane bits 0..1 as DPP-folded min and max (bound_ctrl) + a select on the lane mask: 3 VALU,
    # no compare in VCC, instead of v_sub_co_u32_dpp / s_xor / v_cndmask_b32_dpp (+1%)
    "wqpmm": [("consensus_wide.hip", """  else if constexpr (M == 1) BCE_DPP_STAGE8_ANY("quad_perm:[1,0,3,2]", FLIP);
  else if constexpr (M == 2) BCE_DPP_STAGE8_ANY("quad_perm:[2,3,0,1]", FLIP);
  else if constexpr (M == 3) BCE_DPP_STAGE8_ANY("quad_perm:[3,2,1,0]", FLIP);""", """  else {
    constexpr int CT = (M == 1) ? 0xB1 : (M == 2) ? 0x4E : 0x1B;
    const bool lo_lane = (lower >> lane_id()) & 1;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)key[FLIP ? 7 - r : r], CT, 0xF, 0xF, true);
      const unsigned mn = min(key[r], y), mx = max(key[r], y);
      o[r] = lo_lane ? mn : mx;
    }
  }""")],
    # (the 6-wave bin -- two workgroups per CU at 4 waves/SIMD -- with its probabilities loaded
    # late to free 16 VGPRs, alone or at 5 waves/SIMD for three workgroups per CU (13 dwords
    # still spilled), also with the 3-wave bin: 1.352 / 1.471 / 1.476 vs 1.345 ms,
    # profiles/r03x/ab.txt; not kept)
    # longest bins strictly first (round 2/3 order; the 6-wave-first order is -1.3%)
    "wordlong": [("consensus.hip", "static const int kOrder[BCE_NBINS] = {12, 10, 11, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};",
                  "static const int kOrder[BCE_NBINS] = {12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};")],
    # (also moving the 3-wave bin before the 4-wave bin: no further change)
    # the 1537..2048 bin (4-wave workgroups) on the side stream, launched with the 6-wave bin
    # first on st: 2 x 6 + 1 x 4 waves fill a CU's 16 wave slots (+8.5%: 1.443 vs 1.329 ms)
    "wside4": [("consensus.hip", "static const int kOrder[BCE_NBINS] = {12, 10, 11, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};",
                "static const int kOrder[BCE_NBINS] = {12, 10, 9, 11, 8, 7, 6, 5, 4, 3, 2, 1, 0};"),
               ("consensus.hip", "hipStream_t sb = (b <= side_last) ? side : st;",
                "hipStream_t sb = (b <= side_last || (b == 9 && !merge_np2)) ? side : st;")],
    # (FAST runs inside one thread's R sorted positions averaged in phase 3 -- their sum from
    # the registers, the average over the leader's sorted slot -- so the per-unique phase reads
    # one slot: +6%, 1.41 vs 1.33 ms, parity green, profiles/r03aa/ab.txt; not kept)
    # (the 2049..3072 bin split at 2560 -- markets <= 2560 on 5-wave workgroups, three per CU
    # -- measured 1.379 vs 1.329 ms, parity green, profiles/r03ac/ab.txt; not kept.  Neither
    # were the non-power-of-two bins split out of EXACT's power-of-two launches again:
    # 2.149 vs 2.024 ms, profiles/r03ab/ab.txt)
    # (a FAST dedup-before-sort path -- LDS hash of sids with CAS inserts, a prefix count for
    # the unique index, 64-bit fixed-point atomic sums, then only the u distinct keys sorted,
    # on half the network when u <= P/2 -- was correct (wide/consensus parity green) but
    # 2.27 vs 1.32 ms: contended LDS atomics on hot sources, ten barriers per market and
    # 10-34 spilled VGPRs; profiles/r03ad/ab.txt, not kept)
    # FAST duplicate runs summed by the whole wave from 24 / 96 signals instead of 48
    # (24: same, 96: +1%, profiles/r03af/ab.txt)
    "wrun24": [("consensus_wide.hip", "constexpr int kWaveRun = 48;", "constexpr int kWaveRun = 24;")],
    "wrun96": [("consensus_wide.hip", "constexpr int kWaveRun = 48;", "constexpr int kWaveRun = 96;")],
    # LDS-DMA helpers that save and restore M0 around the DMA (the compiler ignores an M0
    # clobber: M0 is reserved); written in round 3, not yet run on a GPU (tools/gpu_r03aj.sh)
    "wm0save": [("consensus_common.hpp",
                 'asm volatile("s_mov_b32 m0, %0\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %1, off" ::"s"(l), "v"(g) : "memory", "m0");',
                 'uint32_t keep;\n  asm volatile("s_mov_b32 %0, m0\\n\\ts_mov_b32 m0, %1\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %2, off\\n\\ts_mov_b32 m0, %0" : "=&s"(keep) : "s"(l), "v"(g) : "memory");'),
                ("consensus_common.hpp",
                 'asm volatile("s_mov_b32 m0, %0\\n\\ts_nop 0\\n\\tglobal_load_lds_dword %1, off" ::"s"(l), "v"(g) : "memory", "m0");',
                 'uint32_t keep;\n  asm volatile("s_mov_b32 %0, m0\\n\\ts_mov_b32 m0, %1\\n\\ts_nop 0\\n\\tglobal_load_lds_dword %2, off\\n\\ts_mov_b32 m0, %0" : "=&s"(keep) : "s"(l), "v"(g) : "memory");')],
    # ---- exact-preserving ablations: a compare-exchange stage applied twice is a no-op on
    # the data, so these time one class of sort stages without changing the results
    "xin2": [("consensus_wide.hip", """        key[r] = x < y ? x : y;
        key[r2] = x < y ? y : x;""", """        unsigned a1 = x < y ? x : y, b1 = x < y ? y : x;
        asm volatile("" : "+v"(a1), "+v"(b1));
        key[r] = a1 < b1 ? a1 : b1;
        key[r2] = a1 < b1 ? b1 : a1;""")],
    "xlane2": [("consensus_wide.hip", "      dpp_stage8<MK, flip>(key, (uint64_t)ballot(lower));\n",
                "      dpp_stage8<MK, flip>(key, (uint64_t)ballot(lower));\n      dpp_stage8<MK, flip>(key, (uint64_t)ballot(lower));\n"),
               ("consensus_wide.hip", """    for (int r = 0; r < R; ++r) key[r] = ((key[r] < y[r]) == lower) ? key[r] : y[r];
  } else {""", """    for (int r = 0; r < R; ++r) key[r] = ((key[r] < y[r]) == lower) ? key[r] : y[r];
#pragma unroll
    for (int r = 0; r < R; ++r) y[r] = lane_xor<MK>(key[flip ? R - 1 - r : r]);
#pragma unroll
    for (int r = 0; r < R; ++r) key[r] = ((key[r] < y[r]) == lower) ? key[r] : y[r];
  } else {""")],
    "xxw2": [("consensus_wide.hip", """      for (int r = 0; r < R; ++r) key[r] = max(key[r], y[flip ? R - 1 - r : r]);
    }
  }
  if constexpr (J > 1)""", """      for (int r = 0; r < R; ++r) key[r] = max(key[r], y[flip ? R - 1 - r : r]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; r += 4)
      *reinterpret_cast<uint4*>(buf + (r >> 2) * PL + t * 4) = make_uint4(key[r], key[r + 1], key[r + 2], key[r + 3]);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; r += 4) {
      const uint4 y4 = real ? *reinterpret_cast<const uint4*>(buf + (r >> 2) * PL + (t ^ MT) * 4)
                            : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
      y[r] = y4.x;
      y[r + 1] = y4.y;
      y[r + 2] = y4.z;
      y[r + 3] = y4.w;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const unsigned yr = y[flip ? R - 1 - r : r];
      key[r] = ((key[r] < yr) == lower) ? key[r] : yr;
    }
  }
  if constexpr (J > 1)""")],
    # one extra workgroup barrier per stage on the wave-crossing stages only (no LDS work)
    "xxwbar": [("consensus_wide.hip", """      for (int r = 0; r < R; ++r) key[r] = max(key[r], y[flip ? R - 1 - r : r]);
    }
  }
  if constexpr (J > 1)""", """      for (int r = 0; r < R; ++r) key[r] = max(key[r], y[flip ? R - 1 - r : r]);
    }
    __syncthreads();
  }
  if constexpr (J > 1)""")],
    # ---- ablations (timing only; outputs are wrong by construction) ----
    # the sort network run twice (the second pass on sorted keys costs the same)
    "xsort2": [("consensus_wide.hip", "    wide_sort<NN, NW, R>(key, sX, t, lane);\n",
                "    wide_sort<NN, NW, R>(key, sX, t, lane);\n    wide_sort<NN, NW, R>(key, sX, t, lane);\n")],
    # no relconf / present-bit gathers (constant rows)
    "xnogather": [("consensus_wide.hip", "rc[i] = a.relconf[sids[i]];", "rc[i] = make_double2(0.5 + 1e-9 * sids[i], 0.25);"),
                  ("consensus_wide.hip", "pwd[i] = a.pbits[sids[i] >> 5];", "pwd[i] = 0xFFFFFFFFu;")],
    # no normalizedWeight phase
    "xnonw": [("consensus_wide.hip", "    if (a.nweight) {  // core.py:151", "    if (false) {  // core.py:151")],
    # no sorted-probability gather from region A
    "xnosp": [("consensus_wide.hip", "x[r] = (q < n) ? sA[key[r] & QMASK] : 0.0;", "x[r] = (q < n) ? 0.5 : 0.0;")],
    # no run sums (constant averages)
    "xnorun": [("consensus_wide.hip", "avg = (jj < u && len <= kWaveRun) ? run_sum(sA + q0s[i], len) : 0.0;",
                "avg = (jj < u) ? 0.5 : 0.0;")],
}


def build(names):
    tab_variants.build(names, VARIANTS)


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
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        batch.consensus(*d, table, plan=plan, mode=mode, out=res)
        e1.record(st)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    out = {"variant": name, "mode": mode, "median_ms": ms[len(ms) // 2], "min_ms": ms[0]}
    N.check_faults()
    if name == "wprof":  # per workgroup size: share of wave 0's cycles per phase (timed reps only)
        import ctypes
        lib = N.lib()
        buf = (ctypes.c_ulonglong * 128)()
        lib.bce_debug_wprof(buf)  # clear what the ramp accumulated ...
        for _ in range(reps):
            batch.consensus(*d, table, plan=plan, mode=mode, out=res)
        torch.cuda.synchronize()
        lib.bce_debug_wprof(buf)  # ... and read the timed reps
        names = ["keys", "sort", "bar_a", "x+leaders+bar_b", "stores+bar_c", "per_unique", "totals+bar", "nweight"]
        prof = {}
        for nw in range(1, 9):
            v = [buf[nw * 8 + p] for p in range(8)]
            if sum(v):
                prof[f"nw{nw}"] = {k: round(x / sum(v), 4) for k, x in zip(names, v)}
                prof[f"nw{nw}"]["cycles"] = sum(v)
        out["phases"] = prof
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
