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
OUT_DIR = os.path.join(ROOT, "tests", "_build")
# name: (sources, is_reference_program).  Reference programs are compiled unmodified, straight
# from /root/reference; every netcode/ header they include resolves to include/ (this repo).
CPP_CHECKS = {
    "cpp_surface_test": (["tests/cpp/cpp_surface_test.cc"], False),
    "detail_packetizer_test": (["tests/cpp/detail_packetizer_test.cc"], False),
    # bench.py --per-packet: the C-level per-packet workload over libntc.so
    "pp_driver": (["tools/pp_driver.c"], False),
    "ref_cpp_basic": ([REF + "/examples/basic/cpp_basic.cc"], True),
    "ref_c_basic": ([REF + "/examples/basic/c_basic.c"], True),
    "ref_end_to_end": ([REF + "/tests/end_to_end.cc"], True),
    # ctest EndToEnd-MT (tests/CMakeLists.txt:31): encoder and decoder on two threads
    "ref_end_to_end_mt": ([REF + "/tests/end_to_end_mt.cc"], True),
    # the reference's Catch unit tests (ctest UnitTests, tests/CMakeLists.txt:1-29) that compile
    # against this repo's headers; linked with the reference's Catch main (tests/tests.cc)
    "ref_unit_public": ([REF + "/tests/netcode/test_packet.cc", REF + "/tests/netcode/c/test_data.cc",
                         REF + "/tests/netcode/c/test_decoder.cc", REF + "/tests/netcode/test_encoder.cc",
                         REF + "/tests/netcode/test_decoder.cc"], True),
    # the detail layer (include/netcode/detail/*.hh)
    "ref_unit_detail": ([REF + "/tests/netcode/detail/" + f for f in (
        "test_buffer.cc", "test_galois_field.cc", "test_square_matrix.cc", "test_source_list.cc",
        "test_encoder.cc", "test_decoder.cc", "test_invert_matrix.cc", "test_packetizer.cc")]
        + [REF + "/tests/netcode/test_reconstruction.cc"], True),
    # the two suites that need nothing but host code (scalar field ops, detail::invert, the
    # packetizer): also run by the CPU test suite
    "ref_unit_host": ([REF + "/tests/netcode/detail/" + f for f in (
        "test_invert_matrix.cc", "test_packetizer.cc")], True),
}
# Boost is absent from the image.  test_invert_matrix.cc includes <boost/optional/optional_io.hpp>
# (for Catch's printing) and test_packetizer.cc calls boost::endian::native_to_big, which the
# reference's packetizer.hh brings in; tests/boost_shim holds just those two pieces (nothing under
# netcode/), on the include path of the reference Catch suites and force-included there.
BOOST_SHIM = os.path.join(ROOT, "tests", "boost_shim")


def _ref_include_dir() -> str:
    """An include root exposing ONLY the reference's test helpers (tests/, tools/ -- e.g.
    tests/netcode/launch.hh, tools/loss/burst.hh), never its netcode/ library headers: a header
    this repo lacked must fail the build, not silently resolve to the reference's."""
    d = os.path.join(OUT_DIR, "refinc")
    os.makedirs(d, exist_ok=True)
    for sub in ("tests", "tools"):
        link = os.path.join(d, sub)
        if not os.path.islink(link):
            os.symlink(os.path.join(REF, sub), link)
    return d


def _catch_main(verbose: bool) -> str:
    """The reference's Catch main (tests/tests.cc), compiled once (catch.hpp is large)."""
    obj = os.path.join(OUT_DIR, "ref_catch_main.o")
    src = os.path.join(REF, "tests", "tests.cc")
    if not os.path.exists(obj) or os.path.getmtime(obj) < os.path.getmtime(src):
        cmd = ["g++", "-std=c++11", "-O1", "-DCATCH_CONFIG_NO_POSIX_SIGNALS", "-I", REF + "/ext",
               "-c", "-o", obj, src]
        if verbose:
            print("[netcode_amd.build]", " ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    return obj


def build_cpp_checks(verbose: bool = True) -> list[str]:
    os.makedirs(OUT_DIR, exist_ok=True)
    lib_dir = HERE
    built = []
    for name, (srcs, is_ref) in CPP_CHECKS.items():
        srcs_p = [s if os.path.isabs(s) else os.path.join(ROOT, s) for s in srcs]
        if not all(os.path.exists(s) for s in srcs_p):
            continue
        out = os.path.join(OUT_DIR, name)
        deps = srcs_p + [os.path.join(HERE, "libntc.so"), os.path.abspath(__file__)]
        for d in ("include/netcode", "include/netcode/detail", "include/netcode/c",
                  "tests/boost_shim/boost/optional", "tests/boost_shim/boost/endian"):
            dd = os.path.join(ROOT, d)
            deps += [os.path.join(dd, f) for f in os.listdir(dd)]
        if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps if os.path.exists(d)):
            built.append(out)
            continue
        c = srcs_p[0].endswith(".c")
        catch = name.startswith("ref_unit")
        cmd = ["gcc" if c else "g++", "-std=c11" if c else "-std=c++11", "-O1" if catch else "-O2",
               "-Wall", "-I", os.path.join(ROOT, "include")]
        if is_ref:
            cmd += ["-I", _ref_include_dir()]
        if catch:
            cmd += ["-DCATCH_CONFIG_NO_POSIX_SIGNALS", "-I", REF + "/ext", "-I", BOOST_SHIM,
                    "-include", "boost/endian/conversion.hpp"]
        cmd += ["-o", out] + srcs_p
        if catch:
            cmd.append(_catch_main(verbose))
        cmd += ["-L", lib_dir, "-lntc", "-lntc_gf256", "-pthread",
                "-Wl,-rpath," + os.path.relpath(lib_dir, OUT_DIR).join(["$ORIGIN/", ""])]
        if verbose:
            print("[netcode_amd.build]", " ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        built.append(out)
    return built


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_cpp_checks()
