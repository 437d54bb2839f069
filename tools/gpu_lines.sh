#!/bin/bash
# Bench lines on the GPU box (repo root), one step per argument, stopping at the first failure:
#   tools/gpu_lines.sh <tag> [name=bench args]... [pytest=<pytest args>] [smoke=] [sq:<name>=bench args]
#   name=ARGS      timeout 300 python3 bench.py ARGS > gpurun_out/<tag>/<name>.json
#   pytest=ARGS    python -m pytest ARGS (-x -v, 120 s per test) > gpurun_out/<tag>/pytest.txt
#   smoke=         __graft_entry__.smoke() > gpurun_out/<tag>/smoke.txt
#   sq:NAME=ARGS   SQ counters of bench ARGS (tools/gpu_sq.sh), summary -> <tag>/NAME_sq_counters.txt
#   prof:NAME=KERNEL|META|ARGS   rocprof stats + PMC (tools/gpu_profile.sh) -> <tag>/NAME_*.json
#   py:NAME=SCRIPT ARGS  timeout 600 python3 SCRIPT ARGS > gpurun_out/<tag>/NAME.json (a tools/ probe)
#   env:NAME=K=V.. -- ARGS  bench ARGS with environment K=V .. (A/B hooks) -> <tag>/NAME.json
#   trace:NAME=[K=V.. -- ]ARGS  rocprofv3 --kernel-trace of bench ARGS -> <tag>/NAME_bursts.jsonl (tools/trace_bursts.py)
# (replaces round 4's one-off gpu_r04*.sh scripts, verdict r04 item 7)
set -u
tag=$1; shift
o=gpurun_out/$tag
mkdir -p $o
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%=*}; args=${step#*=}
  echo "[gpu_lines] $(date +%T) $name" >&2
  case $name in
    pytest) timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread $args > $o/pytest.txt 2>&1 || exit $? ;;
    smoke) timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $o/smoke.txt 2>&1 || exit $? ;;
    sq:*) n=${name#sq:}; bash tools/gpu_sq.sh ${tag}_$n -- $args || exit $?
          cp gpurun_out/sq_${tag}_$n/summary.txt $o/${n}_sq_counters.txt ;;
    prof:*) n=${name#prof:}; IFS='|' read -r kern meta bargs <<< "$args"
            bash tools/gpu_profile.sh ${tag}_$n "$kern" $meta -- $bargs || exit $?
            for f in stats_summary.json pmc.json kernel_stats.csv; do cp gpurun_out/prof_${tag}_$n/$f $o/${n}_$f 2>/dev/null; done ;;
    trace:*) n=${name#trace:}; vars=X=1
          case "$args" in *" -- "*) vars=${args%% -- *}; args=${args#* -- } ;; esac
          timeout -k 10 600 env $vars rocprofv3 --kernel-trace -d $o/tr_$n -o run --output-format csv -- python3 bench.py $args \
            > $o/$n.log 2>&1 || exit $?
          python3 tools/trace_bursts.py $o/tr_$n > $o/${n}_bursts.jsonl || exit $?
          find $o/tr_$n -name '*.csv' -size +512k -delete ;;
    env:*) n=${name#env:}; vars=${args%% -- *}; bargs=${args#* -- }
          timeout -k 10 300 env $vars python3 bench.py $bargs > $o/$n.json 2> $o/$n.err || exit $? ;;
    py:*) n=${name#py:}; timeout -k 10 600 python3 -u $args > $o/$n.json 2> $o/$n.err || exit $? ;;
    *) timeout -k 10 300 python3 bench.py $args > $o/$name.json 2> $o/$name.err || exit $? ;;
  esac
done
