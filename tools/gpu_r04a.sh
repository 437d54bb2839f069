#!/bin/bash
# Round 4, first GPU call (GPU box, repo root): the whole -m gpu suite after the M0
# save/restore, tie-break fences and MFMA precondition changes; smoke; then rocprof stats +
# FETCH/WRITE passes for the kernels whose profiles were stale (C4 replay_step, C5 fast:
# MFMA + fixup) and SQ counters for the tie-break kernel.
set -u
o=gpurun_out/r04a
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $o/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $o/smoke.txt 2>&1 && \
bash tools/gpu_profile.sh c4 replay_step_kernel sources_this_rank=10000000 -- --config c4 && \
bash tools/gpu_profile.sh c5fast reestimate_votes_mfma_kernel markets_this_rank=1000000 mode=fast -- \
  --config c5 --mode fast --steps 2 --warmup 1 && \
for k in reestimate_fixup_kernel reestimate_agreement_votes_kernel reestimate_consensus_votes_kernel reestimate_total_kernel; do
  python3 tools/pmc_summary.py stats gpurun_out/prof_c5fast/stats $k > gpurun_out/prof_c5fast/stats_$k.json
  python3 tools/pmc_summary.py pmc gpurun_out/prof_c5fast/fetch gpurun_out/prof_c5fast/write $k \
    gpurun_out/prof_c5fast/pmc_$k.json markets_this_rank=1000000 || true
done && \
bash tools/gpu_sq.sh tb -- --config tb
