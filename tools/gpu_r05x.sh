#!/bin/bash
# Round 5: kernel timeline of C3 shard steps (rank 0 and rank 7 of 8) and a full C3 FAST step.
set -u
o=gpurun_out/r05x
mkdir -p $o
export TMPDIR=/tmp
for s in 0 7; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $o/tr_shard$s -o run --output-format csv -- \
    python3 bench.py --config c3 --shard $s/8 --shard-only --prewarm-s 0 --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $o/shard$s.log 2>&1 || exit $?
  python3 tools/step_trace.py $o/tr_shard$s 24 > $o/shard${s}_trace.txt || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/tr_full -o run --output-format csv -- \
  python3 bench.py --config c3 --single-mode --no-cpu-baseline --no-parity --steps 3 --warmup 1 > $o/full.log 2>&1 || exit $?
python3 tools/step_trace.py $o/tr_full 30 > $o/full_trace.txt
find $o -name 'run_*.csv' -size +512k -delete
