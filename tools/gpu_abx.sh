#!/bin/bash
set -o pipefail
tools/gpu_trace_table.sh tt3 || exit 1
tools/gpu_ab.sh ab_slice_noov "UMAMD_WGRAD_OVERLAP=0 UMAMD_BN_SLICE=1" "UMAMD_WGRAD_OVERLAP=0 UMAMD_BN_SLICE=0"
