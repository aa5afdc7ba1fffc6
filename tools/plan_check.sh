#!/bin/bash
# Planner's choice ("auto") against hand-picked plans on the bench workloads.
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/plan_check.jsonl; : > $o
run() { echo "{\"case\": \"$1\"}" >> $o; shift; timeout -k 10 300 python3 tools/plan_sweep.py "$@" >> $o 2>&1; }
run 1080p_sad --cost sad --plans "13,3,0,256,0;13,3,0,256,1;13,16,1,256,1"
run 1080p_ssd --cost ssd --plans "13,3,0,256,0"
run 4k_sad --cost sad --width 3840 --height 2160 --span 64 --plans "13,8,4,256,1;13,4,0,256,1"
run 4k_ssd --cost ssd --width 3840 --height 2160 --span 64 --plans "13,3,0,256,0;13,8,4,256,0"
run 8k_sad --cost sad --width 7680 --height 4320 --blk 8 --span 128 --iters 5 --plans "13,13,0,256,1;13,8,4,256,1"
run 8k_ssd --cost ssd --width 7680 --height 4320 --blk 8 --span 128 --iters 5 --plans "13,9,4,256,0"
cat $o
