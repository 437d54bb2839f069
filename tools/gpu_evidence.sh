#!/bin/bash
# Round evidence on the GPU box (run from the repo root): GPU tests, headline bench with
# the CPU baseline, rocprofv3 kernel stats + HBM PMC for the headline kernel, and the
# secondary configs' bench lines + kernel stats.  Stops at the first crash/timeout.
# Usage: tools/gpu_evidence.sh <tag>
set -u
tag=$1
o=gpurun_out/ev_$tag
mkdir -p $o
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh \
  "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1" \
  "timeout -k 10 300 python bench.py > $o/bench_c2.json 2> $o/bench_c2.err" \
  "tools/gpu_profile_c2.sh $tag consensus_pipe_kernel" \
  "timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $o/bench_c3.json 2> $o/bench_c3.err" \
  "timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $o/bench_c4.json 2> $o/bench_c4.err" \
  "timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline > $o/bench_c5.json 2> $o/bench_c5.err" \
  "cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$o/prof_c3 -o run --output-format csv -- python3 $R/bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 1 > $R/$o/prof_c3.log 2>&1" \
  "cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$o/prof_c4 -o run --output-format csv -- python3 $R/bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 1 > $R/$o/prof_c4.log 2>&1" \
  "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$o/prof_c5 -o run --output-format csv -- python3 $R/bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > $R/$o/prof_c5.log 2>&1"
