#!/bin/bash
# Round 5: parity of the consensus paths touched this round; the small-call bin-merge A/B on
# C3 (full batch + the 8 market shards: nomerge = round-4 launch plan, merge6); the C2 spill
# change A/B (round-4 library vs this tree, same box, twice) with this tree's rocprof + PMC;
# the sort A/B microbenchmark; large-table lines; FAST-only SQ counters of the C3 wide kernels.
set -u
V=tools/bin/variants
mkdir -p gpurun_out/r05c
bash tools/gpu_lines.sh r05c "pytest=tests/test_gpu_wide.py tests/test_gpu_sharded.py tests/test_gpu_consensus.py -q" && \
for v in ship nomerge merge6; do
  L=bayesian-consensus-engine_amd/lib/libbce_hip.so; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05c "c3_$v=--config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-parity --single-mode" "c3sh_$v=--config c3 --shard all/8 --steps 30 --warmup 5" || exit $?
done && \
for i in 1 2; do for v in base ship; do
  L=bayesian-consensus-engine_amd/lib/libbce_hip.so; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05c "c2_${v}_$i=--no-secondary --no-cpu-baseline --steps 200 --warmup 50" || exit $?
done; done && \
timeout -k 10 300 tools/bin/sort_ab > gpurun_out/r05c/sort_ab.json 2> gpurun_out/r05c/sort_ab.err && \
bash tools/gpu_lines.sh r05c "prof:c2=consensus_tab32_kernel|markets=1000000 signals_per_market=32 sources=10000 kernel=consensus_tab32_kernel|--no-secondary" \
  "c3_S2M=--config c3 --steps 20 --warmup 3 --c3-sources 2000000" \
  "c3_S10M=--config c3 --steps 20 --warmup 3 --c3-sources 10000000" \
  "c2_S1M=--sources 1000000 --steps 100 --warmup 10 --no-secondary" \
  "sq:c3f=--config c3 --single-mode --mode fast --no-parity"
