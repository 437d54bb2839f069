#!/bin/bash
# rocprofv3 evidence for the headline kernel (run on the GPU box, from the repo root):
# kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes.
# Usage: tools/gpu_profile_c2.sh <tag> <kernel-substring> [extra bench args...]
set -u
tag=$1; kern=$2; shift 2
export TMPDIR=/tmp
o=gpurun_out/prof_$tag
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/stats -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 20 "$@" > $o/stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $o/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $o/write.log 2>&1 || exit $?
python3 tools/pmc_summary.py stats $o/stats "$kern" > $o/stats_summary.json
python3 tools/pmc_summary.py pmc $o/fetch $o/write "$kern" $o/pmc.json markets=1000000 signals_per_market=32
