#!/bin/bash
# A/B whole-step throughput under knob settings: tools/sweep.sh OUT "ENV1" "ENV2" ...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out/$OUT
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr ' =' '_:' )
  env $cfg timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-roofline --steps 30 > gpurun_out/$OUT/sw_$tag.json 2> gpurun_out/$OUT/sw_$tag.err || { echo "FAILED $cfg"; tail -5 gpurun_out/$OUT/sw_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/$OUT/sw_$tag.json "$cfg"
done
