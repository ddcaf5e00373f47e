#!/bin/bash
# Profile every FB15k config under the PARALLEL schedule (bench + rocprofv3 stats + PMC).
# usage (on the GPU box): tools/gpu_profile_all.sh <tag> [configs...]
set -o pipefail
TAG=${1:-r04}; shift
CFGS=${@:-transe_fb15k transh_fb15k transr_fb15k}
cd "$(dirname "$0")/.."
for C in $CFGS; do
  bash tools/gpu_profile.sh "${TAG}_$C" parallel --config "$C" || exit 1
done
echo all done
