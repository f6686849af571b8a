#!/bin/bash
# whole-step A/B only: tools/gpu_sweep_only.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=$1; shift
bash tools/sweep.sh $TAG "$@"
