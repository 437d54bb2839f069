#!/bin/bash
# Round 5: the sort A/B microbenchmark (tools/sort_ab.hip), large-table lines (C3 at 2M / 10M
# sources, C2 at 1M sources), and FAST-only SQ counters of the C3 wide kernels.
set -u
mkdir -p gpurun_out/r05c
timeout -k 10 300 tools/bin/sort_ab > gpurun_out/r05c/sort_ab.json 2> gpurun_out/r05c/sort_ab.err && \
bash tools/gpu_lines.sh r05c "c3_S2M=--config c3 --steps 20 --warmup 3 --c3-sources 2000000" \
  "c3_S10M=--config c3 --steps 20 --warmup 3 --c3-sources 10000000" \
  "c2_S1M=--sources 1000000 --steps 100 --warmup 10 --no-secondary" \
  "sq:c3f=--config c3 --single-mode --mode fast --no-parity"
