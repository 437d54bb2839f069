#!/usr/bin/env python3
"""Summarise rocprofv3 output for one kernel (experiment tooling, not product code).

  python tools/pmc_summary.py stats <dir> <kernel-substring> [last]
      average duration (ms) from the *kernel_stats.csv of a --kernel-trace --stats run (and of
      the last `last` dispatches in the kernel trace: the timed steps)
  python tools/pmc_summary.py span <dir> <kernel-substring> <kernels-per-step>
      per-step span (first start to last end, ms) of a multi-kernel step from the kernel trace:
      the matching dispatches in start order, chunked by kernels-per-step (side-stream kernels
      overlap the main stream's, so per-kernel averages do not add up to the step)
  python tools/pmc_summary.py pmc <fetch-dir> <write-dir> <kernel-substring> <out.json> [k=v ...]
      (steps_total=N: sum every matching dispatch and divide by N -- per step of a
      multi-kernel config -- instead of averaging per dispatch)
      HBM bytes per launch from two separate --pmc passes (FETCH_SIZE, WRITE_SIZE), corrected
      as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KB) reports 1/2 of the bytes of a
      wide coalesced read on gfx950 -> x2; WRITE_SIZE (KB) is exact for 16-B streaming stores.
      (stream_read_bytes=B: the kernel also gathers.  tools/fetch_calib.hip measured a random
      16-B gather at 64 B of FETCH_SIZE, i.e. counted in full (profiles/archive/r03_fetch_calib.txt),
      so only the B bytes of coalesced streaming reads are under-counted: read = FETCH + B/2.
      Gathers served by the Infinity Cache are counted too, so this is an upper bound on HBM
      reads for a table that stays MALL-resident.)
"""
import csv
import glob
import json
import os
import sys


def _rows(d, pattern):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not files:
        raise SystemExit(f"no {pattern} under {d}")
    out = []
    for f in files:
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def stats(d, kern):
    """(avg ms, calls, full name) of the kernel matching `kern` with the most total time, and
    every matching kernel's row (a substring can match several instantiations)."""
    rows = [r for r in _rows(d, "*kernel_stats.csv") if kern in r["Name"]]
    if not rows:
        raise SystemExit(f"kernel {kern} not in stats")
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    every = [{"kernel": r["Name"], "avg_ms": float(r["AverageNs"]) / 1e6, "min_ms": float(r["MinNs"]) / 1e6,
              "max_ms": float(r["MaxNs"]) / 1e6, "calls": int(r["Calls"])} for r in rows]
    r = rows[0]
    return float(r["AverageNs"]) / 1e6, int(r["Calls"]), r["Name"], every


def steady(d, name, last):
    """Average duration (ms) of the last `last` dispatches of the kernel named exactly `name`
    in the trace: the timed steps, without the clock ramp and warmup dispatches the --stats
    average includes."""
    rows = [r for r in _rows(d, "*kernel_trace.csv") if r["Kernel_Name"] == name]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[-last:]]
    return sum(durs) / len(durs) if durs else None


def counter(d, kern, name, per_step=None):
    vals = [float(r["Counter_Value"]) for r in _rows(d, "*counter_collection.csv")
            if kern in r.get("Kernel_Name", "") and r.get("Counter_Name") == name]
    if not vals:
        raise SystemExit(f"no {name} for {kern} under {d}")
    if per_step:  # several kernels per step (planned launches): total / number of steps
        return sum(vals) / per_step, len(vals)
    vals = vals[1:] if len(vals) > 2 else vals  # drop the cold first launch
    return sum(vals) / len(vals), len(vals)


def span(d, kern, per_step):
    rows = [r for r in _rows(d, "*kernel_trace.csv") if kern in r["Kernel_Name"] and "table_pack" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = []
    for i in range(0, len(rows) - per_step + 1, per_step):
        ch = rows[i:i + per_step]
        if len({r["Kernel_Name"] for r in ch}) != per_step:
            raise SystemExit(f"step {i // per_step}: kernels do not chunk by {per_step}")
        out.append((max(int(r["End_Timestamp"]) for r in ch) - min(int(r["Start_Timestamp"]) for r in ch)) / 1e6)
    srt = sorted(out)
    return {"kernel_substring": kern, "kernels_per_step": per_step, "steps": len(out),
            "median_span_ms": srt[len(srt) // 2], "mean_span_ms": sum(out) / len(out),
            "mean_span_ms_last_50": sum(out[-50:]) / len(out[-50:])}


def main():
    if sys.argv[1] == "span":
        print(json.dumps(span(sys.argv[2], sys.argv[3], int(sys.argv[4]))))
        return
    if sys.argv[1] == "stats":
        ms, calls, name, every = stats(sys.argv[2], sys.argv[3])
        out = {"kernel": name, "avg_ms": ms, "calls": calls}
        if len(sys.argv) > 4:  # the timed steps alone (of that same kernel)
            out[f"avg_ms_last_{sys.argv[4]}"] = steady(sys.argv[2], name, int(sys.argv[4]))
        if len(every) > 1:
            out["matching_kernels"] = every
        print(json.dumps(out))
        return
    fdir, wdir, kern, out = sys.argv[2:6]
    meta = {}
    for kv in sys.argv[6:]:
        if kv.startswith("--meta"):
            continue
        k, v = kv.split("=", 1)
        meta[k] = int(v) if v.isdigit() else v
    per_step = meta.pop("steps_total", None)
    stream_rd = meta.pop("stream_read_bytes", None)
    f_kb, nf = counter(fdir, kern, "FETCH_SIZE", per_step)
    w_kb, nw = counter(wdir, kern, "WRITE_SIZE", per_step)
    if stream_rd is None:
        rd = 2.0 * f_kb * 1024.0
        corr = "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE as is"
    else:
        rd = f_kb * 1024.0 + 0.5 * float(stream_rd)
        corr = (f"FETCH_SIZE + half of the {stream_rd} streamed read bytes (gathers counted in full, "
                "profiles/archive/r03_fetch_calib.txt), WRITE_SIZE as is")
    wr = w_kb * 1024.0
    j = dict(meta, kernel=kern, fetch_size_kb=f_kb, write_size_kb=w_kb, launches=[nf, nw],
             read_bytes_corrected=rd, write_bytes=wr, hbm_bytes_per_launch=rd + wr, correction=corr)
    with open(out, "w") as fh:
        json.dump(j, fh, indent=1)
    print(json.dumps(j))


if __name__ == "__main__":
    main()
