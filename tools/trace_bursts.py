"""Per-burst kernel summary of a rocprofv3 --kernel-trace run (e.g. `bench.py --shard all/8
--shard-only`, which times every rank's shard in turn): dispatches are split into bursts at
idle gaps longer than --gap ms (host work between shards), and for each burst the mean
duration of every kernel, its dispatch count and queue, and the mean step span (first to last
dispatch of one repetition of the burst's kernel sequence) are printed as JSON lines, with each
kernel's mean start / end (t0_us / t1_us) relative to its repetition's first dispatch.
  python3 tools/trace_bursts.py <rocprof output dir> [--gap 20] [--filter bce::]"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap", type=float, default=20.0)
    ap.add_argument("--filter", default="bce::")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if a.filter in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    bursts, cur, last_end = [], [], None
    for r in rows:
        s = int(r["Start_Timestamp"])
        if last_end is not None and s - last_end > a.gap * 1e6:
            bursts.append(cur)
            cur = []
        cur.append(r)
        last_end = max(last_end or 0, int(r["End_Timestamp"]))
    if cur:
        bursts.append(cur)
    for i, b in enumerate(bursts):
        per = defaultdict(list)
        q, wgs = {}, defaultdict(int)
        for r in b:
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void bce::", "").split("(")[0]
            per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            q[name] = r.get("Queue_Id", r.get("Stream_Id", "?"))
            try:
                wgs[name] = max(wgs[name], int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1))
            except (KeyError, ValueError):
                pass
        # repetitions are delimited by the kernel that repeats most often, the earliest such
        # (one-off setup kernels such as a table pack do not delimit)
        cnt = defaultdict(int)
        for r in b:
            cnt[r["Kernel_Name"]] += 1
        top = max(cnt.values())
        first = next(r["Kernel_Name"] for r in b if cnt[r["Kernel_Name"]] == top)
        starts = [int(r["Start_Timestamp"]) for r in b if r["Kernel_Name"] == first]
        steps = len(starts)
        # span of each repetition: from one start of the first kernel to the next
        spans = [(starts[k + 1] - starts[k]) / 1e3 for k in range(len(starts) - 1)]
        # mean start / end of each kernel relative to its repetition's first dispatch (the
        # overlap of the side stream's kernels with the main stream's)
        import bisect
        offs = defaultdict(list)
        for r in b:
            k = bisect.bisect_right(starts, int(r["Start_Timestamp"])) - 1
            if 0 <= k < len(starts) - 1:
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void bce::", "").split("(")[0]
                offs[name].append(((int(r["Start_Timestamp"]) - starts[k]) / 1e3, (int(r["End_Timestamp"]) - starts[k]) / 1e3))
        out = {"burst": i, "dispatches": len(b), "steps": steps,
               "step_us_median": sorted(spans)[len(spans) // 2] if spans else None,
               "kernels": {k: {"n": len(v), "mean_us": round(sum(v) / len(v), 2), "queue": q[k], "max_wgs": wgs[k],
                               "t0_us": round(sum(x[0] for x in offs[k]) / len(offs[k]), 1) if offs[k] else None,
                               "t1_us": round(sum(x[1] for x in offs[k]) / len(offs[k]), 1) if offs[k] else None}
                           for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
