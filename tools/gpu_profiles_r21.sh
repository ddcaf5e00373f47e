#!/bin/bash
# Round-4 profiles: K4 (the bench default: TransR n=50 FB15k-shaped) and K5
# (TransR n=100, 1M entities), each bench line + rocprofv3 kernel trace + PMC passes.
set -o pipefail
bash tools/gpu_profile.sh r21 parallel --late-epoch 0 && \
bash tools/gpu_profile.sh r21 parallel --config transr_k5 --only --no-cpu-baseline --no-epoch
