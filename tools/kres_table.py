"""Summarise -Rpass-analysis=kernel-resource-usage output: one line per kernel
(demangled-ish template args, VGPRs, spills, occupancy)."""
import re
import sys

cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    n = r["name"]
    t = re.search(r"I(L.*)EEvNS", n)
    args = re.findall(r"L([ib])(\d+)E", t.group(1)) if t else []
    print(f"{n.split('hpgq')[1][2:22]:20s} <{','.join(v for _, v in args)}> VGPR {r.get('VGPRs')} "
          f"spillV {r.get('VGPRs Spill')} spillS {r.get('SGPRs Spill')} occ {r.get('Occupancy')}")
