"""The built gfx950 code of libhpgq, disassembled on the CPU (no GPU): the
segmented engine kernels keep the properties DESIGN.md §4.1 measured.

Round 5 found that two rare LDS adds had become FLAT atomics (their pointer
went through an empty asm and came out generic); a FLAT operation that may be
in flight makes hipcc's wait-count pass wait for EVERY load at each later use,
all through the unit loop.  Round 5 kept that accident in the single-end stats
/ filter kernel (C2), which measured faster with the coarse waits; round 6
states C2's wait explicitly in the source (tri_body, PF) and every segmented
kernel must carry no FLAT load or atomic.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hpg-fastq_amd", "libhpgq.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _tools():
    return (os.path.exists(LIB) and shutil.which("objcopy")
            and os.path.exists(os.path.join(LLVM, "clang-offload-bundler"))
            and os.path.exists(os.path.join(LLVM, "llvm-objdump")))


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    """{demangled-ish kernel symbol: [instruction mnemonics]} over every gfx950
    code object of libhpgq.so (the .hip_fatbin section holds one offload
    bundle per translation unit, back to back)."""
    if not _tools():
        pytest.skip("libhpgq.so or the LLVM offload tools are missing")
    d = tmp_path_factory.mktemp("isa")
    fat = d / "fatbin.bin"
    # (an explicit output file: without one objcopy rewrites its input in place,
    # under every other test that has libhpgq.so mapped)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", LIB, str(d / "copy.so")], check=True,
                   capture_output=True)
    blob = fat.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    assert starts, "no offload bundle in .hip_fatbin"
    out = {}
    for i, s in enumerate(starts):
        part = d / f"b{i}.bin"
        part.write_bytes(blob[s:starts[i + 1] if i + 1 < len(starts) else len(blob)])
        co = d / f"b{i}.o"
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                            f"--targets={TARGET}", f"--input={part}", f"--output={co}"], capture_output=True)
        if r.returncode or not co.exists() or co.stat().st_size == 0:
            continue
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", str(co)], check=True,
                             capture_output=True, text=True).stdout
        cur = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                cur = m.group(1)
                out.setdefault(cur, [])
                continue
            m = re.match(r"^\s+([a-z_][a-z0-9_]*)\s", line)
            if cur and m:
                out[cur].append(m.group(1))
    assert out, "no gfx950 code disassembled"
    return out


def _segmented(kernels):
    # engine_tri_kernel<MINW, NM, EDIT, G, FOLLOW> / engine_tri_x_kernel<MINW, NM, G, FOLLOW, XM, EDIT>
    return {k: v for k, v in kernels.items() if "engine_tri_kernel" in k or "engine_tri_x_kernel" in k}


def test_every_geometry_and_variant_is_in_the_library(kernels):
    seg = _segmented(kernels)
    # 3 geometries x (SE/PE x stats/edit) first stages + the x-kernels + wide follow-ups
    assert len(seg) >= 30, sorted(seg)


def test_no_flat_memory_ops_in_any_segmented_kernel(kernels):
    """Round 5 found two rare LDS adds compiled as FLAT atomics (their pointer
    went through an empty asm and came out generic), which made hipcc wait for
    every load at each use; C2 kept them on purpose.  Round 6 states C2's
    coarse wait explicitly (an s_waitcnt in tri_body) and no segmented kernel
    may carry a FLAT load or atomic."""
    bad = {}
    for name, ops in _segmented(kernels).items():
        # (the follow-up stages' one flat_store is the host-mapped deferral
        # report, written once before the loop and waited for at once)
        n = sum(op.startswith(("flat_load", "flat_atomic")) for op in ops)
        if n:
            bad[name] = n
    assert not bad, bad
