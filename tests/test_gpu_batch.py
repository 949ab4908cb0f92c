"""GPU tests of the online batching adaptor (netcode/c/ext.h ntc_batch_*):
encoders attached to a batch emit, at flush time, exactly the packet sequence their unbatched twins
emit immediately -- across field sizes, code types, windows, acks that shrink the window while
repairs are pending, and detaching mid-stream."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi(gpu):
    from netcode_amd import capi as c
    c.load()
    return c


CONFIGS = [
    # w, systematic, rate, window
    (8, True, 4, 32), (8, True, 3, None), (8, False, 5, 8), (16, True, 2, 10), (4, True, 6, 12),
    (32, False, 3, 5),
]


def _make(capi, w, systematic, rate, window):
    e = capi.Encoder(w)
    e.set_rate(rate)
    e.set_code_type(systematic)
    if window:
        e.set_window_size(window)
    return e


def test_batched_encoders_match_unbatched(capi, oracle):
    rng = np.random.default_rng(7)
    batch = capi.Batch()
    pairs = []
    for cfg in CONFIGS:
        a, b = _make(capi, *cfg), _make(capi, *cfg)
        a.set_batch(batch)
        pairs.append((cfg, a, b))
    flushes = 0
    for step in range(120):
        for cfg, a, b in pairs:
            w = cfg[0]
            n = int(rng.integers(1, 400)) * (4 if w >= 16 else 1)
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            a.add_data(data)
            b.add_data(data)
            if step % 11 == 10:
                a.generate_repair()
                b.generate_repair()
            for c in capi.Encoder.COUNTERS:          # state updates immediately
                assert getattr(a, c) == getattr(b, c), c
        if step % 17 == 16:                          # an ack from a decoder that saw b's packets
            cfg, a, b = pairs[0]
            dec = oracle.Decoder(in_order=False)
            for p in b.packets[-20:]:
                dec.add_packet(p)
            dec.generate_ack()
            assert a.add_packet(dec.packets[-1]) == b.add_packet(dec.packets[-1])
            assert a.window == b.window
        if rng.random() < 0.2:
            assert batch.pending > 0
            batch.flush()
            flushes += 1
            assert batch.pending == 0
            for cfg, a, b in pairs:
                assert a.packets == b.packets, cfg
    batch.flush()
    assert flushes > 5
    for cfg, a, b in pairs:
        assert a.packets == b.packets, cfg
        assert len(a.packets) > 100


def test_detach_flushes_and_delete_discards(capi):
    batch = capi.Batch()
    a, b, c = capi.Encoder(), capi.Encoder(), capi.Encoder()
    for e in (a, c):
        e.set_rate(2)
        e.set_batch(batch)
    b.set_rate(2)
    for i in range(7):
        d = bytes([i]) * (10 + i)
        for e in (a, b, c):
            e.add_data(d)
    assert a.packets == [] and batch.pending > 0
    a.set_batch(None)                 # flushes the batch: a (and c) catch up
    assert a.packets == b.packets and c.packets == b.packets
    for e in (a, b, c):
        e.add_data(b"tail")
    assert a.packets == b.packets     # detached: immediate again
    n_before = len(c.packets)
    assert batch.pending > 0
    e = None                          # (the loop variable still referenced c)
    del c                             # an attached encoder's queued packets are discarded
    assert batch.pending == 0
    batch.flush()
    assert len(b.packets) > n_before
