#!/bin/bash
set -o pipefail
tools/gpu_trace_table.sh tt2 || exit 1
tools/gpu_ab.sh ab_wflush "UMAMD_WGRAD_FLUSH_GFLOP=0" "UMAMD_WGRAD_FLUSH_GFLOP=40" || exit 1
tools/gpu_ab.sh ab_wflush2 "UMAMD_WGRAD_FLUSH_GFLOP=20" "UMAMD_WGRAD_FLUSH_GFLOP=80"
