#!/bin/bash
# Round-4 profiles: K4 (the bench default: TransR n=50 FB15k-shaped) and K5
# (TransR n=100, 1M entities), each bench line + rocprofv3 kernel trace + PMC passes,
# into gpurun_out/prof_r21_k4 and gpurun_out/prof_r21_k5.
# usage: tools/gpu_profiles_r21.sh [k4|k5|both]
set -o pipefail
W=${1:-both}
if [ "$W" != k5 ]; then bash tools/gpu_profile.sh r21_k4 parallel --late-epoch 0 || exit 1; fi
if [ "$W" != k4 ]; then bash tools/gpu_profile.sh r21_k5 parallel --config transr_k5 --only --no-cpu-baseline --no-epoch || exit 1; fi
