#!/usr/bin/env python3
"""Per-kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage
output (stdin): name, VGPRs, AGPRs, SGPRs, spills, scratch, occupancy."""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    k, _, v = m.group(1).strip().partition(": ")
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    n = r["name"]
    try:
        n = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        pass
    print(f"{r.get('VGPRs','?'):>4} v {r.get('AGPRs','?'):>3} a {r.get('SGPRs','?'):>4} s "
          f"spill s{r.get('SGPRs Spill','?'):>4} v{r.get('VGPRs Spill','?'):>3} "
          f"scr {r.get('ScratchSize [bytes/lane]','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?'):>2}  {n}")
