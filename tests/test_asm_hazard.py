"""The store-data hazard, checked in the shipped gfx950 code.

A VMEM store of more than 8 bytes (global / buffer / flat / scratch
dwordx3 / dwordx4, and the 128-bit-data cmpswap_x2 atomics) reads its data
VGPRs over two cycles: a VALU instruction that writes one of them within 2
wait states of the store overwrites the data first.  hipcc pads its own
stores; it does not know an inline-asm statement is such a store, so the
split fast kernel's asm stores (nsd_kernels.hip st_b128 / put_rec_st) end
in `s_nop 1` inside the string.  Without it a depth-3 build wrote corrupt
list entries and faulted the GPU (round 3, commit 06a13b0).

This test disassembles every gfx950 code object of libnsdissect.so
(llvm-objcopy .hip_fatbin -> clang-offload-bundler -> llvm-objdump) and
walks, from every such store, every control-flow path (branches followed)
until 2 wait states have passed: no VALU write to the store's data VGPRs
may come first.  A checker self-test feeds it a listing with the hazard."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "netsniff-ng_amd", "libnsdissect.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TOOLS = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
NEED = 2   # wait states between a > 8-byte VMEM store and a VALU write of its data VGPRs

STORE = re.compile(r"^(global|buffer|flat|scratch)_(store_dwordx[34]|atomic_cmpswap_x2)")
LINE = re.compile(r"^\s+(\S+)\s*([^/]*?)\s*//\s*([0-9A-Fa-f]+):")


def vregs(op):
    op = op.strip()
    m = re.match(r"v\[(\d+):(\d+)\]$", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()


def parse(listing):
    """[(addr, mnemonic, operands)] of every instruction of an llvm-objdump -d
    listing, and addr -> index."""
    ins = []
    for line in listing.splitlines():
        m = LINE.match(line)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return ins, {a: k for k, (a, _, _) in enumerate(ins)}


def violations(listing):
    """Stores whose data VGPRs a VALU write reaches within NEED wait states,
    on any path: [(store address, store text, writer address, writer text)]."""
    ins, at = parse(listing)
    bad = []
    for i, (addr, mn, ops) in enumerate(ins):
        if not STORE.match(mn):
            continue
        parts = [p.strip() for p in ops.split(",")]
        # global / flat / scratch: vaddr, vdata, ...; buffer: vdata, vaddr, ...
        data = vregs(parts[0] if mn.startswith("buffer") else parts[1])
        assert data, (hex(addr), mn, ops)
        stack, seen = [(i + 1, 0)], set()
        while stack:
            k, ws = stack.pop()
            if ws >= NEED or k >= len(ins) or (k, ws) in seen:
                continue
            seen.add((k, ws))
            a2, m2, o2 = ins[k]
            if m2.startswith("v_") and vregs(o2.split(",")[0]) & data:
                bad.append((hex(addr), f"{mn} {ops}", hex(a2), f"{m2} {o2}"))
                continue
            if m2 == "s_nop":
                step = int(o2.split()[0], 0) + 1 if o2.strip() else 1
            else:
                step = 1
            if m2 in ("s_endpgm", "s_setpc_b64"):
                continue
            if m2.startswith("s_branch") or m2.startswith("s_cbranch"):
                off = int(o2.split()[0], 0)
                off = off - 65536 if off >= 32768 else off
                tgt = a2 + 4 + 4 * off
                if tgt in at:
                    stack.append((at[tgt], ws + step))
                if m2.startswith("s_branch"):
                    continue
            stack.append((k + 1, ws + step))
    return bad


def disassemble(lib, tmp):
    fat = os.path.join(tmp, "fatbin.bin")
    subprocess.run([TOOLS[0], f"--dump-section=.hip_fatbin={fat}", lib], check=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for k, a in enumerate(starts):
        b = starts[k + 1] if k + 1 < len(starts) else len(data)
        part = os.path.join(tmp, f"b{k}.bin")
        open(part, "wb").write(data[a:b])
        co = part + ".co"
        subprocess.run([TOOLS[1], "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        out.append(subprocess.run([TOOLS[2], "-d", co], check=True, capture_output=True, text=True).stdout)
    return out


def test_checker_finds_the_hazard():
    bad = """
	global_store_dwordx4 v[14:15], v[8:11], off nt             // 000000000100: DC7E8000 007F080E
	v_add_u32_e32 v9, 1, v2                                    // 000000000108: 68120481
"""
    padded = bad.replace("	v_add", "	s_nop 1                                                    // 000000000108: BF800001\n	v_add")
    other = bad.replace("v_add_u32_e32 v9", "v_add_u32_e32 v12")
    branched = """
	global_store_dwordx4 v[2:3], v[4:7], off                   // 000000000100: DC708000 007F0402
	s_cbranch_execz 1                                          // 000000000108: BF880001
	s_nop 0                                                    // 00000000010C: BF800000
	v_mov_b32_e32 v6, 0                                        // 000000000110: 7E0C0280
"""
    assert len(violations(bad)) == 1
    assert violations(padded) == [] and violations(other) == []
    assert len(violations(branched)) == 1           # the taken branch skips the nop


@pytest.mark.skipif(not all(os.path.exists(t) for t in TOOLS) or not os.path.exists(LIB),
                    reason="ROCm LLVM tools or the product library missing")
def test_no_store_data_hazard_in_product(tmp_path):
    listings = disassemble(LIB, str(tmp_path))
    assert listings
    stores = sum(len([1 for _, mn, _ in parse(x)[0] if STORE.match(mn)]) for x in listings)
    assert stores > 20                               # the kernels' 16-byte stores are there
    kernels = "".join(listings)
    assert "dissect_fast" in kernels and "dissect_all" in kernels
    bad = [v for x in listings for v in violations(x)]
    assert not bad, bad[:10]
    shutil.rmtree(str(tmp_path), ignore_errors=True)
