"""The bit-sliced MAC jumps into its shared block table by computed addresses: block c at
table + 128 c (tools/gen_bitslice_table.py).  Check, on the assembled device code, that the
generated include is current, that every block label sits where that formula says, that every
block fits its 128 bytes and uses only the registers of the table contract, and that every
kernel's PC-relative computation of the table address lands on the fast or the safe copy -- a
wrong target would send the waves into arbitrary code (CPU-only; needs hipcc)."""
import importlib.util
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"


def _gen():
    spec = importlib.util.spec_from_file_location("gen", os.path.join(ROOT, "tools", "gen_bitslice_table.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g


def test_generated_include_is_current(tmp_path):
    g = _gen()
    inc = os.path.join(ROOT, "netcode_amd", "csrc", "gf_bitslice_table.inc")
    old = open(inc).read()
    g.OUT = str(tmp_path / "table.inc")
    g.main()
    assert open(g.OUT).read() == old, "re-run tools/gen_bitslice_table.py"


def test_blocks_compute_the_field_product():
    """Each block's ops, interpreted on symbolic planes, give plane p of c*x for every c: the
    XOR of the input planes q with bit p of c*alpha^q set."""
    g = _gen()
    lo, hi, stmts = g.table_planes()
    # Y[n] as a bitmask over input planes 0..7
    Y = [1 << q for q in range(8)] + [0] * (g.NPLANES - 8)
    for st in stmts:
        m = re.match(r"Y\[(\d+)\] = Y\[(\d+)\] \^ Y\[(\d+)\];", st)
        Y[int(m.group(1))] = Y[int(m.group(2))] ^ Y[int(m.group(3))]
    for c in range(256):
        acc = [0] * 8
        for op in g.block_ops(c):
            regs = [int(x) for x in re.findall(r"v(\d+)", op)]
            dst, src = regs[0] - g.ACC, regs[2:]
            assert 0 <= dst < 8 and regs[1] == regs[0]
            for r in src:
                assert g.Y0 <= r < g.Y0 + g.NPLANES
                acc[dst] ^= Y[r - g.Y0]
        for p in range(8):
            want = sum(1 << q for q in range(8) if (g.gmul(c, 1 << q) >> p) & 1)
            assert acc[p] == want, (c, p)


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(OBJDUMP)), reason="no ROCm toolchain")
def test_table_layout_and_entry_addresses(tmp_path):
    from netcode_amd.build import DEVFLAGS
    g = _gen()
    src = os.path.join(ROOT, "netcode_amd", "csrc", "ntc_gf256.hip")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I",
                           os.path.join(ROOT, "include"), "--cuda-device-only", "-c", *DEVFLAGS, "-o",
                           str(tmp_path / "k.o"), src], cwd=tmp_path, stderr=subprocess.DEVNULL)
    # the LINKED code object (relocations applied), as it is loaded on the device
    obj = str(tmp_path / "k_gfx950.co")
    subprocess.check_call([BUNDLER, "--unbundle", "--type=o", "--input=" + str(tmp_path / "k.o"),
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + obj])
    syms, data = {}, set()
    for line in subprocess.run([OBJDUMP, "-t", obj], capture_output=True, text=True, check=True).stdout.splitlines():
        parts = line.split()
        if parts and parts[-1].startswith("ntc_bs_"):
            syms[parts[-1]] = int(parts[0], 16)
        elif any(x in parts for x in (".rodata", ".data", ".bss")):
            data.add(int(parts[0], 16))    # data objects other kernels locate the same way
    for tag in ("f", "s"):
        base = syms[f"ntc_bs_{tag}"]
        assert base % 128 == 0
        for c in range(256):
            assert syms[f"ntc_bs_{tag}{c}"] == base + g.BLOCK * c, (tag, c)
        assert syms[f"ntc_bs_ret_{tag}"] == base + 256 * g.BLOCK
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", obj], capture_output=True, text=True, check=True).stdout
    lines = dis.splitlines()
    targets = []
    for i, l in enumerate(lines[:-2]):
        if "s_getpc_b64 s[96:97]" not in l:
            continue
        a = re.search(r"s_add_u32 s96, s96, (0x[0-9a-f]+)\s+// ([0-9A-F]+):", lines[i + 1])
        b = re.search(r"s_addc_u32 s97, s97, (0x[0-9a-f]+|-?\d+)\s+//", lines[i + 2])
        assert a and b, lines[i:i + 3]
        hi = int(b.group(1), 16) if b.group(1).startswith("0x") else int(b.group(1)) & 0xFFFFFFFF
        targets.append((int(a.group(2), 16) + int(a.group(1), 16) + (hi << 32)) & (2**64 - 1))
    # (a PC-relative pair into s[96:97] that lands on a data object, e.g. a plan kernel's
    # constant table, is not a table entry)
    targets = [t for t in targets if t not in data]
    assert len(targets) >= 16, "every bit-sliced MAC kernel locates the table"
    assert all(t in (syms["ntc_bs_f"], syms["ntc_bs_s"]) for t in targets), [hex(t) for t in targets]
    shutil.rmtree(tmp_path, ignore_errors=True)
