#!/bin/bash
# rocprofv3 stats + PMC for every bench line's dominant kernel (GPU box, repo root).  The PMC
# meta keys are what bench.py / bench_extra.py match before using a file's `traffic`.
# steps_total = consensus launches per PMC pass of that bench command (warmup + timed, plus
# the c3 line's other-mode steps), so the C3 figure is per step; stream_read_bytes = the
# streamed (coalesced) read bytes per step, whose FETCH_SIZE alone is doubled -- the table
# gathers are counted in full (profiles/archive/r03_fetch_calib.txt).
# The raw rocprof CSVs (> 512 KB) are deleted on the box at the end: gpurun copies back at most
# 64 MiB of gpurun_out/.
set -u
bash tools/gpu_profile.sh c2 consensus_tab32_kernel markets=1000000 signals_per_market=32 sources=10000 kernel=consensus_tab32_kernel -- --no-secondary && \
bash tools/gpu_profile.sh c4 replay_step_kernel sources_this_rank=10000000 -- --config c4 && \
bash tools/gpu_profile.sh c3 consensus signals_this_rank=100000000 steps_total=7 stream_read_bytes=1201627112 -- --config c3 --single-mode && \
python3 tools/pmc_summary.py span gpurun_out/prof_c3/stats "bce::" 12 > gpurun_out/prof_c3/step_span.json && \
bash tools/gpu_profile.sh c3S10M consensus signals_this_rank=100000000 sources=10000000 steps_total=7 stream_read_bytes=1201627112 -- --config c3 --single-mode --c3-sources 10000000 && \
bash tools/gpu_profile.sh tb "tiebreak_lpm_kernel<true, false, 1, 32, false>" markets=1000000 -- --config tb && \
bash tools/gpu_profile.sh tbr "tiebreak_lpm_kernel<true, false," markets=1000000 ragged=1 steps_total=8 -- --config tb --ragged && \
for c5 in c5:reestimate_consensus_votes_kernel:exact c5mfma:reestimate_votes_mfma_kernel:mfma; do
  IFS=: read -r tag kern md <<< "$c5"
  bash tools/gpu_profile.sh $tag $kern markets_this_rank=1000000 mode=$md -- --config c5 --mode $md --steps 2 --warmup 1 --single-mode && \
  python3 tools/pmc_summary.py stats gpurun_out/prof_$tag/stats reestimate_agreement_votes_kernel > gpurun_out/prof_$tag/stats_agreement.json && \
  python3 tools/pmc_summary.py pmc gpurun_out/prof_$tag/fetch gpurun_out/prof_$tag/write reestimate_agreement_votes_kernel \
    gpurun_out/prof_$tag/pmc_agreement.json markets_this_rank=1000000 || exit $?
done && \
bash tools/gpu_profile.sh ns namespace_resolve_kernel sources=10000000 -- --config ns && \
bash tools/gpu_profile.sh agg aggregate_kernel groups=10000 -- --config agg --single-mode && \
python3 tools/roofline_check.py gpurun_out > gpurun_out/roofline_check.txt && \
find gpurun_out -path 'gpurun_out/prof_*' -name 'run_*.csv' -size +512k -delete
