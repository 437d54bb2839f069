#!/bin/bash
set -u
o=gpurun_out/r03y2
mkdir -p $o
timeout -k 10 500 python3 tools/wide_variants.py run word6 wside4 wbase word6 wside4 wbase --modes fast --reps 20 > $o/ab.txt 2>&1
