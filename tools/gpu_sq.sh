#!/bin/bash
# SQ counters for one bench config (run on the GPU box from the repo root): three --pmc
# passes (at most 8 SQ counters each, MI355X_MICROARCH.md), summed per kernel name.
# Usage: tools/gpu_sq.sh <tag> -- [bench args...]   ->  gpurun_out/sq_<tag>/summary.txt
set -u
tag=$1; shift; [ "$1" = "--" ] && shift
export TMPDIR=/tmp
o=gpurun_out/sq_$tag
mkdir -p $o
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM TA_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $o/p$i -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 "$@" > $o/p$i.log 2>&1 || exit $?
done
python3 - "$o" > $o/summary.txt <<'PY'
import csv, glob, os, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(o, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "bce::" not in k:
            continue
        # drop the namespace before cutting at the argument list: "(anonymous namespace)" holds
        # the first "(" of every kernel in an unnamed namespace
        k = k.replace("(anonymous namespace)::", "").replace("void bce::", "").split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(acc.items()):
    print(k)
    for c in sorted(d):
        print(f"  {c:28s} {d[c]:.4g}")
    if d.get("SQ_BUSY_CYCLES") and d.get("SQ_ACTIVE_INST_VALU"):
        print(f"  valu_active/wave_cycles      {d['SQ_ACTIVE_INST_VALU'] / max(d.get('SQ_WAVE_CYCLES', 1), 1):.3f}")
PY
