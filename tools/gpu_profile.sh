#!/bin/bash
# rocprofv3 evidence for one bench config (run on the GPU box, from the repo root):
# kernel-trace stats of the bench command, then FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes (MI355X_MICROARCH.md: one counter block per pass; FETCH x2 on gfx950).
# Usage: tools/gpu_profile.sh <tag> <kernel-substring> <meta k=v ...> -- [bench args...]
# Output: gpurun_out/prof_<tag>/{stats_summary.json, pmc.json, *.log} (copy pmc.json to
# measurements/ and the summaries to profiles/ afterwards).
set -u
tag=$1; kern=$2; shift 2
meta=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do meta+=("$1"); shift; done
[ $# -gt 0 ] && shift
export TMPDIR=/tmp
o=gpurun_out/prof_$tag
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/stats -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 --prewarm-s 0.5 "$@" > $o/stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --prewarm-s 0 "$@" > $o/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --prewarm-s 0 "$@" > $o/write.log 2>&1 || exit $?
python3 tools/pmc_summary.py stats $o/stats "$kern" 50 > $o/stats_summary.json
cp $o/stats/run_kernel_stats.csv $o/kernel_stats.csv 2>/dev/null || find $o/stats -name '*kernel_stats.csv' -exec cp {} $o/kernel_stats.csv \;
python3 tools/pmc_summary.py pmc $o/fetch $o/write "$kern" $o/pmc.json "${meta[@]}"
