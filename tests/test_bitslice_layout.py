"""The bit-sliced MAC jumps into its block tables by precomputed offsets (site * kBjSite +
kBjVo[v], tools/gen_bitslice_chain.py).  Assemble the device code and check that every block label
of every chain instance sits exactly where that formula says (CPU-only; needs hipcc)."""
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
    spec = importlib.util.spec_from_file_location("gen", os.path.join(ROOT, "tools", "gen_bitslice_chain.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g


def test_generated_include_is_current(tmp_path):
    g = _gen()
    inc = os.path.join(ROOT, "netcode_amd", "csrc", "gf_bitslice_chain.inc")
    old = open(inc).read()
    g.OUT = str(tmp_path / "chain.inc")
    g.main()
    assert open(g.OUT).read() == old, "re-run tools/gen_bitslice_chain.py"


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(OBJDUMP)), reason="no ROCm toolchain")
def test_block_addresses_match_offsets(tmp_path):
    from netcode_amd.build import DEVFLAGS
    g = _gen()
    src = os.path.join(ROOT, "netcode_amd", "csrc", "ntc_gf256.hip")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                           "--cuda-device-only", "-c", "-save-temps", *DEVFLAGS, "-o", str(tmp_path / "k.o"), src],
                          cwd=tmp_path, stderr=subprocess.DEVNULL)
    obj = [f for f in os.listdir(tmp_path) if f.endswith("gfx950.o")][0]
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(tmp_path / obj)], capture_output=True,
                         text=True, check=True).stdout
    labs = {m.group(2): int(m.group(1), 16)
            for m in re.finditer(r"^([0-9a-f]+) <(L[A-Za-z0-9_]+)>:", dis, re.M)}
    checked = 0
    for name, addr in labs.items():
        m = re.match(r"L([fs])(\d+)_(\d+)_(\d+)$", name)
        if not m:
            continue
        tag, site, v, inst = m.group(1), int(m.group(2)), int(m.group(3)), m.group(4)
        base = labs[("Ltf" if tag == "f" else "Lts") + inst]
        assert addr == base + site * g.SITE + g.VO[v], name
        checked += 1
    assert checked > 1000
    shutil.rmtree(tmp_path, ignore_errors=True)


def _gidx_gen():
    spec = importlib.util.spec_from_file_location("gengx", os.path.join(ROOT, "tools", "gen_bitslice_gidx.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g


def test_gidx_include_is_current(tmp_path):
    g = _gidx_gen()
    inc = os.path.join(ROOT, "netcode_amd", "csrc", "gf_bitslice_gidx.inc")
    old = open(inc).read()
    g.OUT = str(tmp_path / "gidx.inc")
    g.main()
    assert open(g.OUT).read() == old, "re-run tools/gen_bitslice_gidx.py"


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(OBJDUMP)), reason="no ROCm toolchain")
def test_shared_table_layout_and_entry_addresses(tmp_path):
    """The shared-table chains (gf_bitslice_gidx.inc): block c of the out-of-kernel table sits at
    table + 128 c, and every kernel's PC-relative computation of the table address (getpc + lo +
    hi, a negative offset: the table precedes the kernels) lands exactly on ntc_gx3_f /
    ntc_gx3_s -- a wrong target would send the waves into arbitrary code."""
    from netcode_amd.build import DEVFLAGS
    src = os.path.join(ROOT, "netcode_amd", "csrc", "ntc_gf256.hip")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I",
                           os.path.join(ROOT, "include"), "--cuda-device-only", "-c", *DEVFLAGS, "-o",
                           str(tmp_path / "k.o"), src], cwd=tmp_path, stderr=subprocess.DEVNULL)
    # the LINKED code object (relocations applied), as it is loaded on the device
    obj = str(tmp_path / "k_gfx950.co")
    subprocess.check_call([BUNDLER, "--unbundle", "--type=o", "--input=" + str(tmp_path / "k.o"),
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + obj])
    syms = {}
    for line in subprocess.run([OBJDUMP, "-t", obj], capture_output=True, text=True, check=True).stdout.splitlines():
        parts = line.split()
        if parts and parts[-1].startswith("ntc_gx3_"):
            syms[parts[-1]] = int(parts[0], 16)
    for tag in ("f", "s"):
        base = syms[f"ntc_gx3_{tag}"]
        for c in range(256):
            assert syms[f"ntc_gx3_{tag}{c}"] == base + 128 * c, (tag, c)
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", obj], capture_output=True, text=True, check=True).stdout
    lines = dis.splitlines()
    targets = []
    for i, l in enumerate(lines[:-2]):
        if "s_getpc_b64 s[96:97]" not in l:
            continue
        a = re.search(r"s_add_u32 s96, s96, (0x[0-9a-f]+)\s+// ([0-9A-F]+):", lines[i + 1])
        b = re.search(r"s_addc_u32 s97, s97, (0x[0-9a-f]+|-?\d+)\s+//", lines[i + 2])
        if not (a and b):
            continue                                  # the in-kernel chains: forward label offsets
        hi = int(b.group(1), 16) if b.group(1).startswith("0x") else int(b.group(1)) & 0xFFFFFFFF
        targets.append((int(a.group(2), 16) + int(a.group(1), 16) + (hi << 32)) & (2**64 - 1))
    assert targets, "no shared-table entry found"
    assert all(t in (syms["ntc_gx3_f"], syms["ntc_gx3_s"]) for t in targets), [hex(t) for t in targets]
    shutil.rmtree(tmp_path, ignore_errors=True)
