#!/usr/bin/env python3
"""Each bench line's roofline `frac` against bytes / the rocprof time of the same profiled
run (experiment tooling, not product code).

  python tools/roofline_check.py [gpurun_out]   -> one row per line, and the worst deviation

For every tools/gpu_profile.sh directory (gpurun_out/prof_<line>/) the bench JSON line that
rocprofv3 --kernel-trace --stats ran is in stats.log; its `bytes_per_launch` divided by the
rocprof time of the same step -- the dominant kernel's average over the timed steps, plus
the other kernels of that step (C5: the agreement kernel; tb: the second launch; C3: the step
span from the kernel trace, side-stream overlap included) -- gives the fraction the line
should report.
"""
import json
import os
import sys

PEAK = 8000.0  # GB/s, MI355X HBM3E (the bench lines' `peak`)


def last_json(path):
    lines = [ln for ln in open(path) if ln.startswith("{")]
    return json.loads(lines[-1])


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    rows, worst = [], 0.0
    for line in ("c2", "c3", "c4", "c5", "tb", "ns", "agg"):
        d = os.path.join(root, f"prof_{line}")
        if not os.path.isdir(d):
            continue
        bench = last_json(os.path.join(d, "stats.log"))
        r = bench["roofline"]
        st = json.load(open(os.path.join(d, "stats_summary.json")))
        if line == "c3":
            span = json.load(open(os.path.join(d, "step_span.json")))
            ms, how = span["mean_span_ms_last_50"], "step span (kernel trace, last 50 steps)"
        else:
            ms, how = st["avg_ms_last_50"], "dominant kernel, last 50 dispatches"
            others = [k for k in st.get("matching_kernels", [])[1:]]
            if line == "c5":
                ag = json.load(open(os.path.join(d, "stats_agreement.json")))
                ms += ag["avg_ms"]
                how += " + agreement kernel average"
            elif others:
                ms += sum(k["avg_ms"] for k in others)
                how += " + the other matching launches' averages"
        want = r["bytes_per_launch"] / (ms * 1e-3) / 1e9 / PEAK
        dev = r["frac"] / want - 1.0
        worst = max(worst, abs(dev))
        rows.append({"line": line, "bench_frac": r["frac"], "bench_avg_launch_ms": r["avg_launch_ms"],
                     "rocprof_ms": ms, "rocprof_basis": how, "bytes_per_launch": r["bytes_per_launch"],
                     "frac_from_rocprof": want, "deviation": dev, "traffic": r.get("traffic")})
    for row in rows:
        print(json.dumps(row))
    print(json.dumps({"worst_abs_deviation": worst, "lines": len(rows)}))


if __name__ == "__main__":
    main()
