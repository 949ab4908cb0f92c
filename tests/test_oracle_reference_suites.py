"""The checker pinned by the reference's OWN tests (CPU, no GPU).

Every GPU parity test compares the HIP engine with the oracle (oracle/ntc_oracle.c).  Here the
oracle itself is held to the expectations the reference's test programs encode: they are compiled
unmodified from /root/reference against tests/oracle_surface/ -- the reference's C++ API as bindings
over the oracle (oracle/build_surface.py) -- and must pass:
  * tests/netcode/detail/test_invert_matrix.cc:123-233 -- inverses equal to the jerasure code the
    test embeds (w = 4/8/16/32), the singular 3x3 reported, M * M^-1 = I;
  * test_galois_field.cc, test_reconstruction.cc:21-276 -- x * 1/x = 1, the worked reconstruction
    examples (sizes and bytes);
  * test_packetizer.cc:34-229 -- ack / repair / source round trips incl. 1024-id and sparse id lists,
    big ids, and the hand-crafted truncated packets (overflow_error at exactly size + 1);
  * detail/test_encoder.cc, detail/test_decoder.cc -- repair building and the decoder's sources /
    repairs / missing sources / counters after every packet, outdated drops, useless repairs,
    failed full decodings, in-order delivery;
  * tests/netcode/test_encoder.cc, test_decoder.cc -- public encoder / decoder: windows, acks, rates,
    the adaptive rate, non-systematic codes, ack periods;
  * tests/end_to_end.cc:50-73 -- its in-order data handler throws on any wrong, missing or
    reordered payload byte; the counters it prints equal SURVEY §6's reference-build counters.
What stays unpinned: the field polynomial's bytes.  The reference holds no byte vectors for its
regions (gf-complete is absent and none of its tests prints a product), so a different irreducible
polynomial would pass these suites too; the SURVEY §8(c) KATs (tests/golden/kat.json) are the only
byte-level anchor."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BUILD = os.path.join(HERE, "_build")
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))


@pytest.fixture(scope="module")
def programs(oracle):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import build_surface
    built = build_surface.build(verbose=False)
    if not built:
        pytest.skip("reference tree absent: the suites are built in the build container only")
    return {os.path.basename(p): p for p in built}


@pytest.mark.parametrize("prog", ["oracle_ref_detail", "oracle_ref_public"])
def test_reference_catch_suites_pass_on_oracle(programs, prog):
    r = subprocess.run([programs[prog]], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "All tests passed" in r.stdout


@pytest.mark.parametrize("n", ["1000", "10000"])
def test_reference_end_to_end_on_oracle(programs, n):
    r = subprocess.run([programs["oracle_ref_end_to_end"], n], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]          # the in-order data check throws otherwise
    got = {}
    for line in r.stdout.splitlines():
        for key, name in (("Sent ", "sent"), ("Lost ", "lost"), ("Received repairs ", "received_repairs"),
                          ("Received sources ", "received_sources"), ("Useless repairs ", "useless_repairs"),
                          ("Decoded ", "decoded"), ("Handled data ", "handled_data")):
            if line.startswith(key):
                got[name] = int(line[len(key):])
    assert got == KAT["end_to_end"][n]
