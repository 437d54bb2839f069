#!/bin/bash
# Round 4: C3 layout x launch-structure A/B (parity-gated), shard predictions per variant,
# and the tie-break stage batching (GPU tests + tb line).
set -u
o=gpurun_out/r04c
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k tiebreak --timeout 120 \
  --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb.json 2> $o/tb.err && \
timeout -k 10 500 python3 tools/wide_variants.py run wbase wnoswz tafter tless --modes fast --reps 20 > $o/ab_team.txt 2>&1 && \
BCE_WIDE_TEAM=0 timeout -k 10 400 python3 tools/wide_variants.py run wbase wnoswz --modes fast --reps 20 > $o/ab_bins.txt 2>&1 && \
for v in wnoswz tafter tless; do
  BCE_LIB=tools/ablate_build/$v/libbce_hip.so timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 20 --warmup 3 > $o/shards_$v.json 2> $o/shards_$v.err || exit 1
done && \
BCE_WIDE_TEAM=0 BCE_LIB=tools/ablate_build/wnoswz/libbce_hip.so timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 20 --warmup 3 > $o/shards_bins_wnoswz.json 2> $o/shards_bins_wnoswz.err
