#!/bin/bash
# Round 4: the all-bins team kernel for C3 + the rotated sorted-probability layout + the
# native JSONL front end -- wide / consensus / drop-in / jsonl parity, C3 A/B (team vs one
# launch per bin), the 8-shard strong-scaling prediction with each, a kernel trace, the layout
# A/B (parity-gated harness), and the f2 front-end throughput.
set -u
o=gpurun_out/r04b
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_consensus.py tests/test_gpu_dropin.py tests/test_gpu_jsonl.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > $o/c3_team.json 2> $o/c3_team.err && \
BCE_WIDE_TEAM=0 timeout -k 10 200 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > $o/c3_bins.json 2> $o/c3_bins.err && \
timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 > $o/c3_shards_team.json 2> $o/c3_shards_team.err && \
BCE_WIDE_TEAM=0 timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 > $o/c3_shards_bins.json 2> $o/c3_shards_bins.err && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- \
  python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-parity > $o/prof.log 2>&1 && \
timeout -k 10 300 python3 tools/bench_jsonl.py --reps 3 > $o/f2_jsonl.json 2> $o/f2_jsonl.err && \
timeout -k 10 400 python3 tools/wide_variants.py run wbase wnoswz --modes fast,exact --reps 20 > $o/swz_ab.txt 2>&1
