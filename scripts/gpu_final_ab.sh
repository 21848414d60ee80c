#!/bin/bash
# End-of-round GPU pass in one call: smoke, every -m gpu test, the bench line
# (CPU baseline), every configuration with its CPU leg, E / R kernel traces and
# the bench's kernel trace + PMC passes.   bash scripts/gpu_final_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_final_a.sh "$1" && bash scripts/gpu_final_b.sh "$1"
