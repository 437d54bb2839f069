#!/bin/bash
# GPU box, repo root: wide/consensus parity on the build with the gather window, A/B of the
# window against the previous loop (whead), then rocprof stats + PMC for C2 and for C3 with
# whichever build was faster.  Stops at the first failing step.
set -u
o=gpurun_out/r03w
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_consensus.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_wide.txt 2>&1 && \
timeout -k 10 400 python3 tools/wide_variants.py run whead wbase wah1 wah3 whead wbase wah1 wah3 --modes fast,exact --reps 20 > $o/ab.txt 2>&1 || exit 1
lib=$(python3 - $o/ab.txt <<'PY'
import json, sys, statistics
r = {}
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        if d["mode"] == "fast":
            r.setdefault(d["variant"], []).append(d["median_ms"])
print("" if statistics.mean(r["wbase"]) <= statistics.mean(r["whead"]) else "tools/ablate_build/whead/libbce_hip.so")
PY
)
echo "c3 profile lib: ${lib:-product}" > $o/choice.txt
bash tools/gpu_profile.sh c2 consensus_tab32_kernel markets=1000000 signals_per_market=32 kernel=consensus_tab32_kernel -- --no-secondary && \
if [ -n "$lib" ]; then export BCE_LIB=$lib; fi && \
bash tools/gpu_profile.sh c3 consensus signals_this_rank=100000000 steps_total=15 -- --config c3
