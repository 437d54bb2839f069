#!/bin/bash
set -u
o=gpurun_out/r03af
mkdir -p $o
timeout -k 10 400 python3 tools/wide_variants.py run wbase wrun24 wrun96 wbase wrun24 wrun96 --modes fast --reps 20 > $o/ab.txt 2>&1
