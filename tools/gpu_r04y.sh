#!/bin/bash
# Round 4: the whole GPU suite + smoke on the final tree.
set -u
o=gpurun_out/r04y
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $o/smoke.txt 2>&1
