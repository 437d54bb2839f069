#!/bin/bash
set -u
o=gpurun_out/r03x
mkdir -p $o
timeout -k 10 500 python3 tools/wide_variants.py run wbase w6late w6late5 w36late5 wqpmm wbase w6late w6late5 w36late5 wqpmm --modes fast --reps 20 > $o/ab.txt 2>&1
