#!/bin/bash
# Round 5: tie-break length buckets -- parity (every tie-break test), the ragged and uniform
# 1M-market lines against the round-4 library on the same box; one C3 shard step's kernel
# trace with the merged small-call plan.
set -u
V=tools/bin/variants
S=bayesian-consensus-engine_amd/lib/libbce_hip.so
export TMPDIR=/tmp
bash tools/gpu_lines.sh r05e "pytest=tests/test_gpu_dropin.py -q -k tiebreak" && \
for v in base ship; do
  L=$S; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05e "tbr_$v=--config tb --ragged --steps 20 --warmup 3" "tb_$v=--config tb --steps 20 --warmup 3 --no-cpu-baseline --no-parity" || exit $?
done && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r05e/trace -o run --output-format csv -- \
  python3 bench.py --config c3 --shard 0/8 --steps 5 --warmup 2 > gpurun_out/r05e/shard0_trace.log 2>&1
