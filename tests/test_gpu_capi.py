"""GPU tests of the per-packet netcode C ABI (libntc.so over the MI355X engine) against the oracle.

Mirrors the reference's own scenarios: examples/basic/c_basic.c, tests/end_to_end.cc (golden
counters), tests/netcode/test_encoder.cc / test_decoder.cc behaviours (window, rate,
non-systematic code, acks, adaptive rate, rejection of wrong packet types), plus randomized
streams compared packet-for-packet and delivery-for-delivery with the oracle.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))


@pytest.fixture(scope="module")
def capi(gpu):
    from netcode_amd import capi as c
    c.load()
    return c


def test_wire_kat(capi):
    k = KAT["wire_rate2_abcd_efghij"]
    enc = capi.Encoder()
    enc.set_rate(k["inputs"]["rate"])
    for d in k["inputs"]["data"]:
        enc.add_data(bytes.fromhex(d))
    assert [p.hex() for p in enc.packets] == k["packets"]


def test_c_basic_scenario(capi):
    # examples/basic/c_basic.c
    enc = capi.Encoder()
    enc.set_window_size(32)
    dec = capi.Decoder(in_order=True)
    dec.set_ack_period_ms(200)
    enc.add_data(b"abc")
    dec.add_packet(enc.packets[-1])
    assert dec.data == [b"abc"]
    enc.add_data(b"defg")
    dec.add_packet(enc.packets[-1])
    assert dec.data == [b"abc", b"defg"] and dec.aligned


@pytest.mark.parametrize("systematic,rate,window,adaptive", [
    (True, 5, None, False), (True, 3, 8, False), (False, 4, 6, False), (True, 2, None, True)])
def test_encoder_packets_match_oracle(capi, oracle, systematic, rate, window, adaptive):
    rng = np.random.default_rng(rate * 7 + (window or 0))
    a, b = capi.Encoder(), oracle.Encoder()
    for e in (a, b):
        e.set_rate(rate)
        e.set_code_type(systematic)
        e.set_adaptive(adaptive)
        if window:
            e.set_window_size(window)
    dec = oracle.Decoder(in_order=False)
    for i in range(60):
        data = rng.integers(0, 256, int(rng.integers(1, 1500)), dtype=np.uint8).tobytes()
        a.add_data(data)
        b.add_data(data)
        if i % 7 == 6:
            a.generate_repair()
            b.generate_repair()
        if i % 10 == 9:                     # ack built by the oracle decoder from what it saw
            for p in b.packets[-12:]:
                if rng.random() > 0.2:
                    dec.add_packet(p)
            dec.generate_ack()
            ack = dec.packets[-1]
            assert a.add_packet(ack) == b.add_packet(ack)
    assert a.packets == b.packets
    assert a.window == b.window and a.rate == b.rate


def test_end_to_end_golden_counters(capi, oracle):
    """tests/end_to_end.cc with 1000 packets through the GPU-backed C ABI."""
    loss = oracle.Burst(95, 5)
    enc, dec = capi.Encoder(), capi.Decoder(in_order=True)
    dec.set_ack_period_ms(0)
    lost = 0
    for i in range(1000):
        e0, d0 = len(enc.packets), len(dec.packets)     # end_to_end.cc:140-144 fresh buffers
        enc.add_data(np.full(256, i, np.uint32).tobytes())
        for p in enc.packets[e0:]:
            if not loss():
                dec.add_packet(p)
            else:
                lost += 1
        if (dec.nb_received_sources + dec.nb_received_repairs) % 50 == 0:
            dec.generate_ack()
            for p in dec.packets[d0:]:                  # incl. acks made by maybe_ack this turn
                if not loss():
                    enc.add_packet(p)
    got = {"sent": 1000, "lost": lost, "received_repairs": dec.nb_received_repairs,
           "received_sources": dec.nb_received_sources, "useless_repairs": dec.nb_useless_repairs,
           "decoded": dec.nb_decoded, "handled_data": len(dec.data)}
    assert got == KAT["end_to_end"]["1000"]
    for i, d in enumerate(dec.data):
        assert d == np.full(256, i, np.uint32).tobytes()


@pytest.mark.parametrize("seed,in_order,p_loss", [(1, True, 0.1), (2, False, 0.25), (3, True, 0.3)])
def test_random_stream_decoder_matches_oracle(capi, oracle, seed, in_order, p_loss):
    """Sliding-window stream with i.i.d. loss and local reordering: the GPU-backed decoder
    delivers the same data in the same order with the same counters as the oracle's restatement
    of detail::decoder."""
    rng = np.random.default_rng(seed)
    enc = oracle.Encoder()
    enc.set_rate(4)
    enc.set_window_size(24)
    for i in range(300):
        enc.add_data(rng.integers(0, 256, int(rng.integers(1, 800)), dtype=np.uint8).tobytes())
    pkts = [p for p in enc.packets if rng.random() >= p_loss]
    for i in range(0, len(pkts) - 3, 5):       # local reordering
        if rng.random() < 0.3:
            pkts[i], pkts[i + 2] = pkts[i + 2], pkts[i]
    a, b = capi.Decoder(in_order=in_order), oracle.Decoder(in_order=in_order)
    for d in (a, b):
        d.set_ack_period_ms(0)
        d.set_ack_nb_packets(128)
    for p in pkts:
        a.add_packet(p)
        b.add_packet(p)
    assert a.data == [d for _, d in b.data]
    for c in capi.Decoder.COUNTERS:
        assert getattr(a, c) == getattr(b, c), c
    assert a.packets == b.packets


def test_rejects_wrong_packet_types(capi):
    enc, dec = capi.Encoder(), capi.Decoder()
    enc.add_data(b"xyz")
    with pytest.raises(capi.NtcError) as e:
        enc.add_packet(enc.packets[0])          # a source given to an encoder
    assert e.value.kind == "packet_type_error"
    with pytest.raises(capi.NtcError) as e:
        dec.add_packet(b"\x07garbage")
    assert e.value.kind == "packet_type_error"
    with pytest.raises(capi.NtcError) as e:
        dec.add_packet(bytes.fromhex("0200000000ffff61"))   # declared length past the end
    assert e.value.kind == "overflow_error"


@pytest.mark.parametrize("mode", ["immediate", "batched", "async", "batched-unpinned", "async-unpinned",
                                  "async-gpunode"])
@pytest.mark.parametrize("flows,items,size,window,rate,loss", [(16, 24, 1024, 32, 4, 10),
                                                               (5, 40, 300, 8, 2, 30),
                                                               (7, 30, 4000, 16, 3, 20)])
def test_c_level_per_packet_matches_oracle(oracle, mode, flows, items, size, window, rate, loss):
    """tools/pp_driver.c (bench.py --per-packet's C-level GPU leg: one encoder / decoder per
    flow through the reference C ABI, immediate, batched or batched with asynchronous flushes)
    produces exactly the packets and the deliveries of the oracle's or_pp_bench on the same payload
    and loss draws -- with the payloads in pinned pool blocks that the device reads and writes
    directly (default) and in malloc'd buffers staged through the flush's copies
    (NTC_BATCH_UNPINNED=1, "-unpinned"); "-gpunode": the pool's slabs from hipHostMalloc instead of
    registered malloc pages (NTC_BATCH_PINNED_NUMA=gpu)."""
    import ctypes as C
    import subprocess
    drv = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "_build",
                       "pp_driver")
    args = [str(x) for x in (flows, items, size, window, rate, loss, 11)]
    env = dict(os.environ)
    if mode.endswith("-unpinned"):
        mode = mode[:-len("-unpinned")]
        env["NTC_BATCH_UNPINNED"] = "1"
    if mode.endswith("-gpunode"):               # pool slabs from hipHostMalloc (the GPU's NUMA node)
        mode = mode[:-len("-gpunode")]
        env["NTC_BATCH_PINNED_NUMA"] = "gpu"
    r = subprocess.run([drv, mode] + args, capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    g = json.loads(r.stdout.strip().splitlines()[-1])
    secs, cnt, hs = (C.c_double * 2)(), (C.c_uint64 * 4)(), (C.c_uint64 * 2)()
    assert oracle.lib().or_pp_bench(flows, items, size, window, rate, loss, C.c_uint64(11), secs, cnt, hs) == 0
    assert [g["packets"], g["received"], g["deliveries"], g["repairs"]] == list(cnt)
    assert g["packets_hash"] == f"{hs[0]:016x}"
    assert g["deliveries_hash"] == f"{hs[1]:016x}"
