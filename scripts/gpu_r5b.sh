#!/bin/bash
# round 5: kernel trace + FETCH/WRITE + SQ/TA/TD counters of the config-2 batch on the lean gather+build path
set -o pipefail
mkdir -p gpurun_out
bash scripts/profile.sh ${1:-r5gb} && bash scripts/pmc_lab.sh ${1:-r5gb} && echo R5B_OK
