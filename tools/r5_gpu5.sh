#!/bin/bash
# round 5: fresh bf16 step trace + backward-order A/B on the current library
set -o pipefail
bash tools/quick_trace.sh r5bf16 || exit 1
bash tools/ab_env.sh r5ord 3 "base:" "defer:OCRK_DEFER_DWX=1" "dxf:OCRK_DX_FIRST=1" || exit 1
