#!/bin/bash
# Round 5: small FAST calls on R = 4 configurations (4-wave 1024-key, 8-wave 2048-key bins)
# -- parity, then the C3 shard A/B against the default configurations, twice.
set -u
V=tools/bin/variants
S=bayesian-consensus-engine_amd/lib/libbce_hip.so
bash tools/gpu_lines.sh r05g "pytest=tests/test_gpu_wide.py tests/test_gpu_sharded.py -q" && \
for i in 1 2; do for v in ship nosmallwide; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05g "c3sh_${v}_$i=--config c3 --shard all/8 --steps 30 --warmup 5" || exit $?
done; done
