#!/bin/bash
# GPU box, repo root: the round-end evidence in one call -- every -m gpu test, smoke(),
# every bench line, rocprof stats + PMC.  Stops at the first failing step.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pt_all.txt 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' \
  > gpurun_out/smoke.txt 2>&1 && \
bash tools/gpu_bench_all.sh && \
bash tools/gpu_prof_all.sh
