#!/bin/bash
# GPU box: T1 A/B (A = lib_ab/ = HEAD, B = lib/ = working tree; 3 alternating
# rounds of scripts/t1_ab.py), then smoke + the GPU suite + the 8K / C5 / C4
# bench lines on B (scripts/gpu_suite.sh).
set -o pipefail
TAG=${1:-r03n}
bash scripts/gpu_ab.sh $TAG/ab 3 || exit 1
bash scripts/gpu_suite.sh $TAG 8k c5 c4
