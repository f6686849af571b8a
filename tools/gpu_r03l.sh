#!/bin/bash
# step table + per-launch trace table + counter passes of the HEAD build
set -o pipefail
T=${1:-r03l}
tools/prof_step.sh ${T}_prof --loader-steps 0 --fp32-steps 0 --no-loss-delta --eager-steps 0 || { echo PROF FAILED; exit 1; }
head -50 gpurun_out/${T}_prof/step_kernels.txt
tools/gpu_pmc_counters.sh ${T}_pmc || { echo PMC FAILED; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/${T}_pmc/counters.json'))
for k,v in d['entries'].items(): print(k, v['launches'], v['mean_us'], v['derived'])
"
