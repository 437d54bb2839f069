#!/bin/bash
# Round 5: parity of the changed consensus paths (4-stream planned call, 64-bit keys, sharded
# runs), then the C3 A/B: round-4 library (base) vs 1 / 2 / 4 planned streams (full batch and
# the 8 market shards).
set -u
V=tools/bin/variants
bash tools/gpu_lines.sh r05b "pytest=tests/test_gpu_wide.py tests/test_gpu_sharded.py tests/test_gpu_consensus.py -q" && \
for v in base ship ps1 ps2; do
  L=bayesian-consensus-engine_amd/lib/libbce_hip.so; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05b "c3_$v=--config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-parity --single-mode" "c3sh_$v=--config c3 --shard all/8 --steps 30 --warmup 5" || exit $?
done
