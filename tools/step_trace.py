"""The last K kernel dispatches of a rocprofv3 --kernel-trace run as a timeline (us from the
first of them): name, start, duration, queue, grid -- for reading one timed step's launch
structure (e.g. a C3 shard step's main / side-stream overlap).
  python3 tools/step_trace.py <rocprof output dir> K [name-substring]"""
import csv
import glob
import os
import sys


def main():
    d, k = sys.argv[1], int(sys.argv[2])
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-k:]
    t0 = int(rows[0]["Start_Timestamp"])
    end = max(int(r["End_Timestamp"]) for r in rows)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void bce::", "").split("(")[0]
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        g = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        print(f"{name[:48]:48s} start {(s - t0) / 1e3:8.1f}  dur {(e - s) / 1e3:7.1f}  queue {q:>3}  grid {g}")
    print(f"span {(end - t0) / 1e3:.1f} us over {len(rows)} dispatches")


if __name__ == "__main__":
    main()
