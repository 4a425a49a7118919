"""Print VGPRs / spills / occupancy of the traversal and shade kernels from
the hipcc -Rpass-analysis=kernel-resource-usage log (lib/obj/wavefront.resources.txt)."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "go-raytracing_amd/lib/obj/wavefront.resources.txt"
cur = None
rows = {}
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    if re.search(r"k_(extend|shadow|shade)ILi8ELb0ELb0ELb[01]E|k_shadeILb[01]ELb0ELb0ELb[01]E", k):
        name = k.replace("_ZN3rtgL", "_ZN3rtg")   # (kernels with internal linkage since round 6)
        print(f"{name[7:40]:34s} vgpr {v.get('VGPRs')} vspill {v.get('VGPRs Spill')} sspill {v.get('SGPRs Spill')} occ {v.get('Occupancy [waves/SIMD]')} scratch {v.get('ScratchSize [bytes/lane]')}")
