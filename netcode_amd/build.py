"""Build the native pieces in-tree (no JIT cache): libntc_gf256.so for gfx950 via hipcc.

The .so lands next to this file so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# Uniform (scalar) branches stay real branches instead of being flattened by the CFG
# structurizer: the bit-sliced MAC dispatches on wave-uniform coefficient nibbles.
DEVFLAGS = ["-mllvm", "-structurizecfg-skip-uniform-regions"]

TARGETS = {
    # GF(2^8) engine: kernels + batched C ABI (include/netcode/gpu.h)
    "libntc_gf256.so": (["csrc/ntc_gf256.hip", "csrc/ntc_dense.hip", "csrc/ntc_wire.hip",
                                          "csrc/ntc_gfw.hip"], []),
    # reference per-packet C ABI (include/netcode/c/*.h) over the engine
    "libntc.so": (["csrc/ntc_capi.cpp"], ["-L", "{here}", "-lntc_gf256", "-Wl,-rpath,$ORIGIN"]),
}


def _stale(out: str, srcs: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = srcs + [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))]
    deps.append(os.path.join(ROOT, "include", "netcode", "gpu.h"))
    cdir = os.path.join(ROOT, "include", "netcode", "c")
    deps += [os.path.join(cdir, f) for f in os.listdir(cdir)]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> list[str]:
    built = []
    for out, (srcs, link) in TARGETS.items():
        out_p = os.path.join(HERE, out)
        srcs_p = [os.path.join(HERE, s) for s in srcs]
        link = [x.replace("{here}", HERE) for x in link]
        if not force and not _stale(out_p, srcs_p):
            built.append(out_p)
            continue
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared"] + DEVFLAGS + [
               "-Wall", "-I", os.path.join(ROOT, "include"), "-o", out_p + ".tmp"] + srcs_p + link
        if verbose:
            print("[netcode_amd.build]", " ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(out_p + ".tmp", out_p)
        built.append(out_p)
    return built


# C++ surface checks (tests/, not product): our own driver of include/netcode/*.hh, and -- when
# the reference tree is present (this container only) -- the reference's own public-API programs
# compiled unmodified against our headers and libntc.so.  Outputs go to tests/_build/ (git-ignored,
# shipped to the GPU box with the tree).
REF = "/root/reference"
CPP_CHECKS = {
    "cpp_surface_test": ("tests/cpp/cpp_surface_test.cc", False),
    "ref_cpp_basic": (REF + "/examples/basic/cpp_basic.cc", True),
    "ref_c_basic": (REF + "/examples/basic/c_basic.c", True),
    "ref_end_to_end": (REF + "/tests/end_to_end.cc", True),
}


def build_cpp_checks(verbose: bool = True) -> list[str]:
    out_dir = os.path.join(ROOT, "tests", "_build")
    os.makedirs(out_dir, exist_ok=True)
    lib_dir = HERE
    built = []
    for name, (src, is_ref) in CPP_CHECKS.items():
        src_p = src if os.path.isabs(src) else os.path.join(ROOT, src)
        if not os.path.exists(src_p):
            continue
        out = os.path.join(out_dir, name)
        deps = [src_p, os.path.join(HERE, "libntc.so")]
        for d in ("include/netcode", "include/netcode/detail", "include/netcode/c"):
            dd = os.path.join(ROOT, d)
            deps += [os.path.join(dd, f) for f in os.listdir(dd)]
        if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps if os.path.exists(d)):
            built.append(out)
            continue
        c = src_p.endswith(".c")
        cmd = ["gcc" if c else "g++", "-std=c11" if c else "-std=c++11", "-O2", "-Wall",
               "-I", os.path.join(ROOT, "include")]
        if is_ref:
            cmd += ["-I", REF]          # only for the reference's own test helpers (tools/loss)
        cmd += ["-o", out, src_p, "-L", lib_dir, "-lntc", "-lntc_gf256",
                "-Wl,-rpath," + os.path.relpath(lib_dir, out_dir).join(["$ORIGIN/", ""])]
        if verbose:
            print("[netcode_amd.build]", " ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        built.append(out)
    return built


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_cpp_checks()
