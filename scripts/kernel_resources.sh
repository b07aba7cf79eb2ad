#!/bin/bash
# usage: scripts/kernel_resources.sh tts-max_amd/csrc/lm_gemm.hip  -> name VGPR spill occupancy
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -c $f -o /tmp/_kr.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -E "Function Name|VGPRs:|VGPRs Spill|Occupancy|LDS Size" | sed -E 's/.*remark: //; s/ \[-Rpass.*//; s/^ +//' \
 | awk '/Function Name/{if(n)print n" | "v" | "sp" | "o" | "l; n=$3; next} /^VGPRs:/{v=$0} /VGPRs Spill/{sp=$0} /Occupancy/{o=$0} /LDS Size/{l=$0} END{print n" | "v" | "sp" | "o" | "l}' \
 | while IFS= read -r line; do name=$(echo "$line" | cut -d' ' -f1); dm=$(echo $name | /opt/rocm/llvm/bin/llvm-cxxfilt 2>/dev/null || echo $name); echo "$dm | ${line#* | }"; done
