#!/bin/bash
set -u
o=gpurun_out/r03ab
mkdir -p $o
timeout -k 10 400 python3 tools/wide_variants.py run wbase wsplitx wbase wsplitx --modes exact --reps 20 > $o/ab.txt 2>&1
