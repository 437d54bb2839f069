#!/bin/bash
# Round 5: parity of the 64-bit-key fused lane stages and the merged small calls; A/Bs on one
# box: 64-bit keys fused vs generic (C3 at 2M / 10M sources), bin merges below 6 vs 3 resident
# rounds (C3 shards), C2 tab kernel (round 4 / late meta (shipped) / early meta), C5 MFMA pass
# register budget (shipped 3 waves/SIMD vs 4 / 5).
set -u
V=tools/bin/variants
S=bayesian-consensus-engine_amd/lib/libbce_hip.so
bash tools/gpu_lines.sh r05d "pytest=tests/test_gpu_wide.py tests/test_gpu_sharded.py -q" && \
for v in ship k64gen; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05d "c3S10M_$v=--config c3 --steps 20 --warmup 3 --c3-sources 10000000 --no-cpu-baseline --no-parity" "c3S2M_$v=--config c3 --steps 20 --warmup 3 --c3-sources 2000000 --no-cpu-baseline --no-parity" || exit $?
done && \
for v in ship merge3; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05d "c3sh_$v=--config c3 --shard all/8 --steps 30 --warmup 5" || exit $?
done && \
for i in 1 2; do for v in base ship tabearly; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05d "c2_${v}_$i=--no-secondary --no-cpu-baseline --steps 300 --warmup 50" || exit $?
done; done && \
for v in ship c5w4 c5w5; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05d "c5_$v=--config c5 --steps 4 --warmup 1 --prewarm-s 0.5 --no-cpu-baseline --no-parity" || exit $?
done
