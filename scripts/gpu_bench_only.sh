#!/bin/bash
# Headline bench only (no CPU baseline): quick A/B of a kernel change (parity must be run separately)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-b}
shift
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bo_$TAG.log 2>&1
rc=$?; echo bench=$rc; exit $rc
