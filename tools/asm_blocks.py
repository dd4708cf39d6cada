"""Per-basic-block instruction counts of one kernel in a hipcc device .s file
(hipcc --cuda-device-only -S): loop depth (from the compiler's block
comments), VALU / SALU / VMEM / LDS counts and the SGPR-spill lane moves, so
the hot loop's body can be read without a profiler.

  python tools/asm_blocks.py /tmp/geo1.s engine_tri_kernelILi3ELi1ELb1 [--min-depth 1]
"""
import argparse
import re

ap = argparse.ArgumentParser()
ap.add_argument("asm")
ap.add_argument("kernel", help="substring of the mangled kernel name")
ap.add_argument("--min-depth", type=int, default=0)
a = ap.parse_args()

lines = open(a.asm).read().splitlines()
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and a.kernel in l)
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+|_Z\w+):", l)
    if m or (cur is None):
        cur = {"name": m.group(1) if m else "entry", "depth": 0, "ins": []}
        blocks.append(cur)
        d = re.search(r"Depth=(\d+)", l)
        if d:
            cur["depth"] = int(d.group(1))
        continue
    if re.match(r"^; %bb\.\d+:", l):   # a fall-through block
        cur = {"name": l.split()[1], "depth": 0, "ins": []}
        d = re.search(r"Depth=(\d+)", l)
        if d:
            cur["depth"] = int(d.group(1))
        blocks.append(cur)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    cur["ins"].append(t.split()[0])


def cls(op):
    if op in ("v_readlane_b32", "v_writelane_b32"):
        return "lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


tot = {}
for b in blocks:
    if b["depth"] < a.min_depth or not b["ins"]:
        continue
    c = {}
    for op in b["ins"]:
        k = cls(op)
        c[k] = c.get(k, 0) + 1
    for k, v in c.items():
        tot[k] = tot.get(k, 0) + v
    print(f"{b['name']:16s} depth {b['depth']}  n {len(b['ins']):4d}  " +
          "  ".join(f"{k} {c.get(k, 0)}" for k in ("valu", "lane", "salu", "vmem", "lds", "wait")))
print("total", tot)
