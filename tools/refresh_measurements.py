"""Copy a tools/gpu_prof_all.sh run into the repo: every gpurun_out/prof_<line>/ summary to
profiles/<tag>/<line>_*, and each line's PMC summary to measurements/pmc_<name>.json (what
bench.py's read_pmc matches before quoting `traffic`; C5 combines its two kernels' bytes).
  python3 tools/refresh_measurements.py <tag>      (after gpurun merged gpurun_out/)"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# prof tag -> measurements file
PMC = {"c2": "pmc_c2.json", "c3": "pmc_c3.json", "c3S10M": "pmc_c3_S10M.json", "c4": "pmc_c4.json",
       "tb": "pmc_tb.json", "tbr": "pmc_tb_ragged.json", "ns": "pmc_ns.json", "agg": "pmc_agg.json"}
# C5: pass 1 + the agreement pass, per mode (the line's own mode is exact)
C5 = {"c5": "pmc_c5.json", "c5mfma": "pmc_c5_mfma.json"}
FILES = ("kernel_stats.csv", "pmc.json", "stats_summary.json", "step_span.json", "pmc_agreement.json",
         "stats_agreement.json")


def main():
    tag = sys.argv[1]
    src, dst = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for line in list(PMC) + list(C5):
        d = os.path.join(src, f"prof_{line}")
        for f in FILES:
            if os.path.exists(os.path.join(d, f)):
                shutil.copy(os.path.join(d, f), os.path.join(dst, f"{line}_{f}"))
    shutil.copy(os.path.join(src, "roofline_check.txt"), os.path.join(dst, "roofline_check.txt"))
    for line, name in PMC.items():
        p = os.path.join(src, f"prof_{line}", "pmc.json")
        if not os.path.exists(p):
            continue
        j = json.load(open(p))
        j["source"] = f"profiles/{tag}/{line}_pmc.json (tools/gpu_prof_all.sh)"
        json.dump(j, open(os.path.join(ROOT, "measurements", name), "w"), indent=1)
    for line, name in C5.items():
        d = os.path.join(src, f"prof_{line}")
        if not os.path.exists(os.path.join(d, "pmc.json")):
            continue
        v = json.load(open(os.path.join(d, "pmc.json")))
        g = json.load(open(os.path.join(d, "pmc_agreement.json")))
        c5 = {"markets_this_rank": v["markets_this_rank"], "mode": v["mode"],
              "kernel": f"{v['kernel']} + {g['kernel']} (one iteration)",
              "hbm_bytes_per_launch": v["hbm_bytes_per_launch"] + g["hbm_bytes_per_launch"],
              "source": f"profiles/{tag}/{line}_pmc.json + profiles/{tag}/{line}_pmc_agreement.json "
                        "(tools/gpu_prof_all.sh)",
              "correction": v.get("correction"), "parts": {"votes": v, "agreement": g}}
        json.dump(c5, open(os.path.join(ROOT, "measurements", name), "w"), indent=1)
    print(f"profiles/{tag}: {len(os.listdir(dst))} files; measurements refreshed")


if __name__ == "__main__":
    main()
