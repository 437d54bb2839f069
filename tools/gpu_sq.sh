#!/bin/bash
# SQ counter passes for the headline kernel (GPU box).  Usage: tools/gpu_sq.sh <tag> [bench args]
set -u
tag=$1; shift
export TMPDIR=/tmp
o=gpurun_out/sq_$tag
mkdir -p $o
timeout -s KILL 60 rocprofv3 -L > $o/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_ACTIVE_INST_SCA,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_INST_LDS,SQ_INST_CYCLES_VMEM_RD,SQ_INST_CYCLES_VMEM_WR,SQ_INSTS_SMEM,GRBM_GUI_ACTIVE,GRBM_COUNT,TA_BUSY_avr,TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } -d $o/p$i -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > $o/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $o/p$i.log; }
done
python3 - "$o" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{o}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "consensus" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):.4g}  (n={len(v)})")
PY
