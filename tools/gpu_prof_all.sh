#!/bin/bash
# rocprofv3 stats + PMC for the headline and the secondary HBM configs (GPU box, repo root).
# steps_total = consensus launches per PMC pass of that bench command (warmup + timed, plus
# the c3 line's other-mode steps), so the PMC figures are per step.
set -u
bash tools/gpu_profile.sh c2 consensus_tab32_kernel markets=1000000 signals_per_market=32 kernel=consensus_tab32_kernel -- --no-secondary && \
bash tools/gpu_profile.sh c4 replay_step_kernel sources_this_rank=10000000 -- --config c4 && \
bash tools/gpu_profile.sh c3 consensus signals_this_rank=100000000 steps_total=15 -- --config c3 && \
bash tools/gpu_profile.sh c5 reestimate markets_this_rank=1000000 steps_total=7 -- --config c5
