#!/bin/bash
# Round record: the -m gpu suite + default bench line + chain counters
# (tools/gpu_round.sh), then rocprofv3 kernel stats + PMC of the TransR and
# TransH FB15k configs (tools/gpu_profile.sh).
set -o pipefail
TAG=${1:-r19}
cd "$(dirname "$0")/.."
bash tools/gpu_round.sh $TAG && bash tools/gpu_profile.sh ${TAG}_transr_fb15k parallel --config transr_fb15k
