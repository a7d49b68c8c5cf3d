#!/bin/bash
# Dev tool: per-kernel VGPR/SGPR/spill/occupancy of the fused resize instances.
cd "$(dirname "$0")/../rust-image-transform_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Icsrc -I../include -c csrc/ik_kernels.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys,re
cur=None
for l in sys.stdin:
    m=re.search(r"remark: +(.*?): (\S+) \[",l)
    if not m: continue
    k,v=m.groups()
    if k=="Function Name": cur=v; out={}
    elif cur and "resize_fused" in cur:
        out[k]=v
        if k=="Occupancy [waves/SIMD]": print(cur[24:60], "vgpr",out.get("VGPRs"),"sgpr",out.get("TotalSGPRs"),"vspill",out.get("VGPRs Spill"),"sspill",out.get("SGPRs Spill"),"occ",v)
'
