"""CPU checks of the header-only C++ surface (include/netcode/{encoder,decoder,packet,data,
errors,dispatch}.hh over libntc.so): it compiles under -std=c++11 with our own driver and -- where
the reference tree is present -- the reference's own public-API programs (examples/basic/
cpp_basic.cc, c_basic.c, tests/end_to_end.cc) compile and link unmodified against it.  Without a
HIP device the programs fail loudly (no CPU fallback)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")


@pytest.fixture(scope="module")
def cpp_checks(native_built):
    from netcode_amd import build
    return {os.path.basename(p): p for p in build.build_cpp_checks(verbose=False)}


def test_own_driver_compiles(cpp_checks):
    assert "cpp_surface_test" in cpp_checks


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference tree not present")
def test_reference_programs_compile_against_our_headers(cpp_checks):
    for name in ("ref_cpp_basic", "ref_c_basic", "ref_end_to_end"):
        assert name in cpp_checks, name


def test_no_device_fails_loudly(cpp_checks):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    r = subprocess.run([cpp_checks["cpp_surface_test"], "10"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "no MI355X engine" in r.stderr


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference tree not present")
def test_reference_host_suites(cpp_checks):
    """The reference's tests/netcode/detail/test_invert_matrix.cc (detail::invert equals the
    embedded jerasure inversion, :123-157; the singular 3x3 fails, :161-180; M * M^-1 = I for
    w = 4/8/16/32, :184-233) and test_packetizer.cc (ack / repair / source round trips, the
    hand-built truncated packets of :160-229), compiled unmodified against include/ with the
    tests-only Boost shim (tests/boost_shim); host code only, so they run here."""
    r = subprocess.run([cpp_checks["ref_unit_host"]], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "All tests passed" in r.stdout, r.stdout[-2000:]


def test_detail_packetizer_cases(cpp_checks):
    """The detail-layer packetizer (include/netcode/detail/packetizer.hh) on the cases of the
    reference's test_packetizer.cc (not buildable here: Boost.Endian) plus the SURVEY §8(c) wire
    KAT; header-only, runs on the CPU."""
    r = subprocess.run([cpp_checks["detail_packetizer_test"]], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout
