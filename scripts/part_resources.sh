#!/bin/bash
# Compile one part of coupling.hip (device only) and print the kernel resource remarks whose
# function name matches a pattern: scripts/part_resources.sh <part 1|2|3> <grep pattern> [extra flags]
part=$1; pat=$2; shift 2
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -c naz_amd/csrc/coupling.hip \
  -o /tmp/part_$part.o -fno-slp-vectorize -DNAZ_PART=$part --offload-device-only \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | grep "remark" | \
  awk -v pat="$pat" '/Function Name/ {show = ($0 ~ pat); if (show) print $NF > "/dev/stderr"} show && /VGPRs|Scratch|Occupancy|AGPRs/ {sub(/.*remark: +/, "  "); print}'
