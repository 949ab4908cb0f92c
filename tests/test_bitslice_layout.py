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
