"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output per kernel (stdin)."""
import re
import sys

cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    keys = ["VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "Occupancy [waves/SIMD]"]
    print(f"{k[:60]:60s} " + " ".join(f"{kk.split()[0]}{'sp' if 'Spill' in kk else ''}={v.get(kk,'-')}" for kk in keys))
