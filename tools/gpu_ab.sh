#!/bin/bash
# Interleaved same-box A/B of library variants through one bench command (GPU box, repo root):
#   tools/gpu_ab.sh <tag> <reps> <variant,variant,...> -- <bench.py args>
# variant "ship" = the in-tree library; any other name = tools/ab/<name>/libbce_hip.so
# (built on the CPU beforehand; tools/ab/ travels with the snapshot, delete it after the A/B).  Every rep runs
# every variant once, in order, into gpurun_out/<tag>/<variant>_<rep>.json; a summary of each
# variant's ms_per_step (and roofline.avg_launch_ms) over the reps lands in <tag>/summary.txt.
# Claim discipline: a change is promoted only when >= 3 interleaved reps beat the
# box-to-box spread.
set -u
tag=$1; reps=$2; variants=$3; shift 3
[ "${1:-}" = "--" ] && shift
o=gpurun_out/$tag
mkdir -p $o
export TMPDIR=/tmp
IFS=',' read -ra VS <<< "$variants"
for rep in $(seq 1 $reps); do
  for v in "${VS[@]}"; do
    if [ "$v" = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/ab/$v/libbce_hip.so; fi
    echo "[gpu_ab] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py "$@" > $o/${v}_$rep.json 2> $o/${v}_$rep.err || exit $?
  done
done
unset BCE_LIB
python3 - "$o" "$variants" "$reps" > $o/summary.txt <<'PY'
import json, sys
o, vs, reps = sys.argv[1], sys.argv[2].split(","), int(sys.argv[3])
for v in vs:
    ms, kl = [], []
    for r in range(1, reps + 1):
        j = json.load(open(f"{o}/{v}_{r}.json"))
        ms.append(j["ms_per_step"])
        kl.append((j.get("roofline") or {}).get("avg_launch_ms"))
    print(f"{v:12s} ms_per_step {' '.join(f'{x:.4f}' for x in ms)}  avg_launch_ms {' '.join(f'{x:.4f}' for x in kl if x)}")
PY
cat $o/summary.txt
