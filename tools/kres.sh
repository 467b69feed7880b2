#!/bin/bash
# Register usage / spills / occupancy of every kernel in one source file:  tools/kres.sh k_ragged.hip
f=${1:-k_ragged.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -c "$(dirname "$0")/../fpnn_amd/csrc/$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' \
 | awk '/Function Name/{n=$3} /^ *VGPRs:/{v=$2} /SGPRs Spill/{ss=$3} /VGPRs Spill/{vs=$3} /Occupancy/{o=$3} /LDS Size/{print n, "vgpr="v, "sgpr_spill="ss, "vgpr_spill="vs, "occ="o}' | c++filt | sed 's/fpnn_aes:://g'
