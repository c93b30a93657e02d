#!/bin/bash
# spill variants: A/B (loose = in-tree, tight, prev) and their SQ/LDS counters
REPS=5 bash tools/gpu_abn.sh tight prev || exit 1
bash tools/exp_pmc_ab.sh tight prev || exit 1
python3 tools/pmc_ab_summary.py default tight prev
