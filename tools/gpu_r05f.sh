#!/bin/bash
# Round 5: the whole GPU suite on this tree; tie-break ragged line with aligned-pair gathers
# (+ rocprof per bucket kernel); C3 shards with / without the second side stream for a small
# call's 65..1024 bins; C5 MFMA on the exact kernel's load schedule vs round 4; C2 PMC.
set -u
V=tools/bin/variants
S=bayesian-consensus-engine_amd/lib/libbce_hip.so
export TMPDIR=/tmp
bash tools/gpu_lines.sh r05f "pytest=tests -m gpu -q" "smoke=" && \
bash tools/gpu_lines.sh r05f "tbr_ship=--config tb --ragged --steps 20 --warmup 3" && \
bash tools/gpu_lines.sh r05f "tbr_contig=--config tb --ragged --steps 20 --warmup 3 --no-cpu-baseline --no-parity --tb-contiguous" && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05f/tbprof -o run --output-format csv -- \
  python3 bench.py --config tb --ragged --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/r05f/tbprof.log 2>&1 && \
for v in ship noside2; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05f "c3sh_$v=--config c3 --shard all/8 --steps 30 --warmup 5" || exit $?
done && \
for v in ship base; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05f "c5_$v=--config c5 --steps 4 --warmup 1 --prewarm-s 0.5 --no-cpu-baseline" || exit $?
done && \
bash tools/gpu_lines.sh r05f "prof:c2=consensus_tab32_kernel|markets=1000000 signals_per_market=32 sources=10000 kernel=consensus_tab32_kernel|--no-secondary"
