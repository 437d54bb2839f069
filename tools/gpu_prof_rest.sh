#!/bin/bash
# The tail of tools/gpu_prof_all.sh (tb, c5, ns, agg + the roofline cross-check), for a pass
# whose first lines already ran.
set -u
bash tools/gpu_profile.sh tb "tiebreak_lpm_kernel<true, false, 1, 32, false>" markets=1000000 -- --config tb && \
bash tools/gpu_profile.sh c5 reestimate_consensus_votes_kernel markets_this_rank=1000000 mode=exact -- --config c5 --steps 2 --warmup 1 --single-mode && \
python3 tools/pmc_summary.py stats gpurun_out/prof_c5/stats reestimate_agreement_votes_kernel > gpurun_out/prof_c5/stats_agreement.json && \
python3 tools/pmc_summary.py pmc gpurun_out/prof_c5/fetch gpurun_out/prof_c5/write reestimate_agreement_votes_kernel \
  gpurun_out/prof_c5/pmc_agreement.json markets_this_rank=1000000 && \
bash tools/gpu_profile.sh c5mfma reestimate_votes_mfma_kernel markets_this_rank=1000000 mode=mfma -- --config c5 --mode mfma --steps 2 --warmup 1 --single-mode && \
bash tools/gpu_profile.sh ns namespace_resolve_kernel sources=10000000 -- --config ns && \
bash tools/gpu_profile.sh agg aggregate_kernel groups=10000 -- --config agg --single-mode && \
python3 tools/roofline_check.py gpurun_out > gpurun_out/roofline_check.txt
