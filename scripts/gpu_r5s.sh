#!/bin/bash
# round 5 (session 2): full GPU suite, then the bench lines of config 2, the request mix and config 4
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5s}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_full.log 2>&1 || { tail -40 gpurun_out/${T}_full.log; exit 1; }
tail -1 gpurun_out/${T}_full.log
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
sum() { python3 -c "
import json,sys
r=json.loads([l for l in open('$1') if l.startswith('{')][-1])
print('$1', round(r['ms_per_step'],4), round(r['roofline']['frac'],4), {k[:18]:v for k,v in r.get('stages_ms',{}).items() if v}, r.get('deferred'))"; }
$B > gpurun_out/${T}_c2.log 2>&1 && sum gpurun_out/${T}_c2.log &&
$B --accept-frac 0.3 --unordered-frac 0.1 > gpurun_out/${T}_mix.log 2>&1 && sum gpurun_out/${T}_mix.log &&
$B --config 4 > gpurun_out/${T}_c4.log 2>&1 && sum gpurun_out/${T}_c4.log
