#!/bin/bash
# Per-kernel register / LDS / occupancy summary of one HIP source (compiler remarks, CPU only).
# Usage: bash tools/resusage.sh cnn_lstm_ctc_ocr_amd/csrc/lstm_persistent.hip [name-filter]
src=${1:?source}
filt=${2:-.}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Icnn_lstm_ctc_ocr_amd/csrc --cuda-device-only \
    -c -o /dev/null "$src" -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *\(.*\) \[-Rpass.*/\1/p' |
  awk -v f="$filt" '/^Function Name:/ {name=$3; keep=(name ~ f); line=""; next}
       keep && /^(VGPRs|AGPRs|Occupancy|LDS Size|VGPRs Spill):/ {line=line " " $0}
       keep && /^LDS Size/ {print substr(name,1,70) ":" line}'
