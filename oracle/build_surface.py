"""TEST INFRASTRUCTURE ONLY: the reference's own test programs compiled against the oracle.

tests/oracle_surface/ restates the reference's C++ API (ntc::encoder / ntc::decoder and the
ntc::detail layer) as thin bindings over oracle/ntc_oracle.c.  This script compiles the reference's
Catch suites and tests/end_to_end.cc -- unmodified, straight from /root/reference -- against that
header set and oracle/libntc_oracle.so, so the checker every GPU parity test trusts is itself held to
the reference's expectations (jerasure-equal inverses, the singular-matrix index, the hand-made
truncated packets, the reconstruction examples, the decoder's state after each packet, the adaptive
rate, the end_to_end in-order content and counters).  The include path holds only
tests/oracle_surface, oracle/ and the reference's tests/ + tools/ (never its netcode/ headers, never
this repo's include/).  Outputs go to tests/_build/ (git-ignored).  Needs /root/reference, so it runs
in the build container only.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "_build")
SURFACE = os.path.join(ROOT, "tests", "oracle_surface")
BOOST_SHIM = os.path.join(ROOT, "tests", "boost_shim")

_D = REF + "/tests/netcode/detail/"
PROGRAMS = {
    # the detail layer: field, inversion (vs the jerasure code embedded in the test), packetizer
    # (hand-crafted truncated packets), repair building, the decoder state machine
    "oracle_ref_detail": [_D + f for f in (
        "test_galois_field.cc", "test_invert_matrix.cc", "test_packetizer.cc", "test_square_matrix.cc",
        "test_source_list.cc", "test_encoder.cc", "test_decoder.cc")]
        + [REF + "/tests/netcode/test_reconstruction.cc"],
    # public ntc::encoder / ntc::decoder: windows, rates, adaptive rate, acks, counters
    "oracle_ref_public": [REF + "/tests/netcode/test_encoder.cc", REF + "/tests/netcode/test_decoder.cc"],
    # tests/end_to_end.cc: 1 KiB payloads, burst loss, in-order content check
    "oracle_ref_end_to_end": [REF + "/tests/end_to_end.cc"],
}


def _refinc() -> str:
    d = os.path.join(OUT, "refinc")
    os.makedirs(d, exist_ok=True)
    for sub in ("tests", "tools"):
        link = os.path.join(d, sub)
        if not os.path.islink(link):
            os.symlink(os.path.join(REF, sub), link)
    return d


def _catch_main(verbose: bool) -> str:
    obj = os.path.join(OUT, "ref_catch_main.o")
    src = os.path.join(REF, "tests", "tests.cc")
    if not os.path.exists(obj) or os.path.getmtime(obj) < os.path.getmtime(src):
        cmd = ["g++", "-std=c++11", "-O1", "-DCATCH_CONFIG_NO_POSIX_SIGNALS", "-I", REF + "/ext", "-c",
               "-o", obj, src]
        if verbose:
            print("[oracle.build_surface]", " ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    return obj


def build(verbose: bool = True) -> list[str]:
    if not os.path.isdir(REF):
        return []
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(HERE, "libntc_oracle.so")
    deps = [lib, os.path.abspath(__file__)]
    for dp, _, fs in os.walk(SURFACE):
        deps += [os.path.join(dp, f) for f in fs]
    built = []
    for name, srcs in PROGRAMS.items():
        out = os.path.join(OUT, name)
        if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps + srcs):
            built.append(out)
            continue
        catch = name != "oracle_ref_end_to_end"
        cmd = ["g++", "-std=c++11", "-O1", "-Wall", "-I", SURFACE, "-I", HERE, "-I", _refinc()]
        if catch:
            cmd += ["-DCATCH_CONFIG_NO_POSIX_SIGNALS", "-I", REF + "/ext", "-I", BOOST_SHIM,
                    "-include", "boost/endian/conversion.hpp"]
        cmd += ["-o", out] + srcs + ([_catch_main(verbose)] if catch else [])
        cmd += [lib, "-pthread", "-Wl,-rpath," + os.path.relpath(HERE, OUT).join(["$ORIGIN/", ""])]
        if verbose:
            print("[oracle.build_surface]", " ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        built.append(out)
    return built


if __name__ == "__main__":
    build()
