#!/bin/bash
# Kernel resource usage (VGPRs, AGPRs, spills, scratch, LDS, occupancy) of one
# source file of the gfx950 library, from the compiler's resource-usage
# remarks:  bash tools/kres.sh csrc/physics/solver.hip [kernel-name-regex]
set -euo pipefail
cd "$(dirname "$0")/../gpu-ecs-madrona_amd"
SRC=$1
RX=${2:-.}
FLAGS="-fno-slp-vectorize"
/opt/rocm/bin/hipcc -std=c++20 -O3 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -ffp-contract=off \
  -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -I../include $FLAGS ${EXTRA:-} \
  --cuda-device-only -c "$SRC" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size|SGPRs:|Spill" |
  sed -e 's/.*remark: //' | awk -v rx="$RX" '/Function Name/ {show = ($0 ~ rx)} show'
