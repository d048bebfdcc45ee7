#!/bin/bash
# Print per-kernel VGPR/AGPR/scratch/occupancy of a HIP source (gfx950).
src=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$src" -o /tmp/_resusage.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 \
 | grep -E "error|Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" \
 | sed -E 's/.*remark: +//; s/ \[-Rpass-analysis=kernel-resource-usage\]//' \
 | awk '/Function Name/{if(line)print line; n=$3; sub(/^_ZN4kite[0-9]+/,"",n); line=substr(n,1,28)} !/Function Name/{line=line" | "$0} END{print line}'
