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
    # deferred (the default): nothing of a goes out before the flush
    assert a.packets == [] and len(b.packets) > 0
    assert batch.pending > 0
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


def _lossy_stream(oracle, w, seed, n=200, p_loss=0.2, rate=4, window=24):
    rng = np.random.default_rng(seed)
    enc = oracle.Encoder(galois_field_size=w)
    enc.set_rate(rate)
    enc.set_window_size(window)
    for i in range(n):
        enc.add_data(rng.integers(0, 256, 4 * int(rng.integers(1, 200)), dtype=np.uint8).tobytes())
    pkts = [p for p in enc.packets if rng.random() >= p_loss]
    for i in range(0, len(pkts) - 3, 5):       # local reordering
        if rng.random() < 0.3:
            pkts[i], pkts[i + 2] = pkts[i + 2], pkts[i]
    return pkts


@pytest.mark.parametrize("w,in_order,seed", [(8, True, 1), (8, False, 2), (16, True, 3), (4, False, 4),
                                             (32, True, 12)])
def test_batched_decoders_match_unbatched(capi, oracle, w, in_order, seed):
    """Deferred (symbolic) decoding: deliveries, acks and counters equal the immediate decoder's and
    the oracle's; the state (counters) advances before the flush, the callbacks at the flush."""
    pkts = _lossy_stream(oracle, w, seed)
    rng = np.random.default_rng(seed + 100)
    batch = capi.Batch()
    a, b = capi.Decoder(w, in_order=in_order), capi.Decoder(w, in_order=in_order)
    o = oracle.Decoder(in_order=in_order, galois_field_size=w)
    for d in (a, b, o):
        d.set_ack_period_ms(0)
        d.set_ack_nb_packets(20)
    a.set_batch(batch)
    for i, p in enumerate(pkts):
        for d in (a, b, o):
            d.add_packet(p)
        for c in capi.Decoder.COUNTERS:
            assert getattr(a, c) == getattr(b, c), c
        if rng.random() < 0.1:
            batch.flush()
            assert a.data == b.data and a.packets == b.packets
    batch.flush()
    assert a.data == b.data == [d for _, d in o.data]
    assert a.packets == b.packets == o.packets
    assert b.nb_decoded > 0


@pytest.mark.parametrize("seed", range(20, 32))
def test_batched_decoders_random_streams(capi, oracle, seed):
    """Random windows (small ones make the decoder drop outdated sources and repairs while reduced
    repairs still name them), repair rates, losses and reorderings, synchronous or asynchronous
    flushes at random points: deliveries and packets equal the oracle's."""
    rng = np.random.default_rng(seed)
    window, rate = int(rng.integers(2, 48)), int(rng.integers(1, 7))
    pkts = _lossy_stream(oracle, 8, seed, n=160, p_loss=float(rng.uniform(0.05, 0.4)), rate=rate,
                         window=window)
    in_order = bool(rng.integers(0, 2))
    batch = capi.Batch(eager=bool(rng.integers(0, 2)), asynchronous=bool(rng.integers(0, 2)))
    a = capi.Decoder(8, in_order=in_order)
    o = oracle.Decoder(in_order=in_order, galois_field_size=8)
    nb = int(rng.integers(4, 64))
    for d in (a, o):
        d.set_ack_period_ms(0)
        d.set_ack_nb_packets(nb)
    a.set_batch(batch)
    for p in pkts:
        a.add_packet(p)
        o.add_packet(p)
        if rng.random() < 0.15:
            batch.flush()
    while True:
        batch.flush()
        if batch.pending == 0:
            break
    assert a.data == [d for _, d in o.data]
    assert a.packets == o.packets


def test_batch_switching_and_shared_batch(capi, oracle):
    """Encoders and decoders on one batch; a decoder leaves batch mode mid-stream (its symbols are
    materialised) and keeps decoding identically."""
    batch = capi.Batch()
    rng = np.random.default_rng(9)
    ea, eb = capi.Encoder(), capi.Encoder()
    for e in (ea, eb):
        e.set_rate(3)
        e.set_window_size(16)
    ea.set_batch(batch)
    da, db = capi.Decoder(in_order=True), capi.Decoder(in_order=True)
    for d in (da, db):
        d.set_ack_period_ms(0)
    da.set_batch(batch)
    sent = 0
    for step in range(150):
        data = rng.integers(0, 256, int(rng.integers(1, 600)), dtype=np.uint8).tobytes()
        ea.add_data(data)
        eb.add_data(data)
        batch.flush()                      # ea's packets appear; da's deliveries for older ones
        assert ea.packets == eb.packets
        for p in eb.packets[sent:]:
            if rng.random() >= 0.2:
                da.add_packet(p)
                db.add_packet(p)
        sent = len(eb.packets)
        if step == 90:
            da.set_batch(None)             # flush + materialise; immediate from here on
    batch.flush()
    assert da.data == db.data and da.packets == db.packets
    assert db.nb_decoded > 0


def test_eager_batch_emits_early_and_reenters(capi):
    """Eager mode (ntc_batch_set_eager): a source packet of an encoder with nothing queued goes out
    inside add_data; the packet handler re-enters a decoder attached to the SAME batch (its
    deliveries and acks are produced during the encoder's call).  Every object's sequence still
    equals its unbatched twin's."""
    batch = capi.Batch(eager=True)
    ea, eb = capi.Encoder(), capi.Encoder()
    da, db = capi.Decoder(in_order=True), capi.Decoder(in_order=True)
    for e in (ea, eb):
        e.set_rate(3)
    for d in (da, db):
        d.set_ack_period_ms(0)
        d.set_ack_nb_packets(7)
    ea.set_batch(batch)
    da.set_batch(batch)
    rng = np.random.default_rng(5)
    drop = set(int(i) for i in rng.choice(400, 60, replace=False))
    seen = {"a": 0, "b": 0}

    def feed(tag, dec):
        def on_packet(pkt):
            i = seen[tag]
            seen[tag] += 1
            if i not in drop:
                dec.add_packet(pkt)       # re-entrant: the decoder shares ea's batch
        return on_packet

    ea._out.on_packet = feed("a", da)
    eb._out.on_packet = feed("b", db)
    early = 0
    for step in range(200):
        data = rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
        n0 = len(ea.packets)
        ea.add_data(data)
        eb.add_data(data)
        early += len(ea.packets) > n0
        if step % 9 == 8:
            while batch.pending:          # events made by callbacks during a flush wait for the next
                batch.flush()
            assert ea.packets == eb.packets
            assert da.data == db.data and da.packets == db.packets
    while batch.pending:
        batch.flush()
    assert early > 0                      # eager: some packets left inside add_data
    assert ea.packets == eb.packets
    assert da.data == db.data and da.packets == db.packets
    assert db.nb_decoded > 0


@pytest.mark.parametrize("eager", [False, True])
def test_async_batch_matches_unbatched(capi, oracle, eager):
    """Asynchronous flushes (ntc_batch_set_async): a flush first delivers the events of the previous
    one, then starts the device work of the queued events and returns; the objects keep producing
    events meanwhile (queued behind the ones in flight).  Encoders and decoders on one batch,
    across field sizes, with the decoders fed from their encoders' packets: every object's packet
    and delivery sequence equals its unbatched twin's once the batch is drained."""
    batch = capi.Batch(eager=eager, asynchronous=True)
    rng = np.random.default_rng(21 + eager)
    flows = []
    for w, rate in ((8, 3), (16, 4), (8, 5), (4, 2)):
        ea, eb = capi.Encoder(w), capi.Encoder(w)
        da, db = capi.Decoder(w, in_order=True), capi.Decoder(w, in_order=True)
        for e in (ea, eb):
            e.set_rate(rate)
            e.set_window_size(24)
        for d in (da, db):
            d.set_ack_period_ms(0)
            d.set_ack_nb_packets(9)
        ea.set_batch(batch)
        da.set_batch(batch)
        flows.append([w, ea, eb, da, db, 0, 0])
    in_flight = 0
    for step in range(160):
        for f in flows:
            w, ea, eb, da, db = f[:5]
            n = int(rng.integers(1, 300)) * (4 if w >= 16 else 1)
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            ea.add_data(data)
            eb.add_data(data)
            # the decoders see what their encoder has emitted so far (b's are all out already)
            for p in ea.packets[f[5]:]:
                if rng.random() >= 0.15:
                    da.add_packet(p)
                    db.add_packet(eb.packets[f[5]])
                f[5] += 1
        if step % 3 == 2:
            batch.flush()
            in_flight += batch.pending > 0
    while batch.pending:
        batch.flush()
    assert in_flight > 10                 # flushes did return with work still in flight
    for w, ea, eb, da, db, _, _ in flows:
        assert ea.packets == eb.packets, w
        assert da.data == db.data and da.packets == db.packets, w
    assert sum(f[4].nb_decoded for f in flows) > 0     # repairs did decode lost sources


def test_async_batch_switch_and_delete_with_work_in_flight(capi, oracle):
    """Asynchronous flushes leave device work in flight: a decoder leaving the batch mid-stream
    drains it first (its deliveries stay in order, then immediate), and a batch deleted with
    events in flight discards them without disturbing a second batch's flushes."""
    rng = np.random.default_rng(31)
    batch = capi.Batch(asynchronous=True)
    ea, eb = capi.Encoder(), capi.Encoder()
    da, db = capi.Decoder(in_order=True), capi.Decoder(in_order=True)
    for e in (ea, eb):
        e.set_rate(3)
        e.set_window_size(16)
    for d in (da, db):
        d.set_ack_period_ms(0)
    ea.set_batch(batch)
    da.set_batch(batch)
    sent = 0
    for step in range(120):
        data = rng.integers(0, 256, int(rng.integers(1, 500)), dtype=np.uint8).tobytes()
        ea.add_data(data)
        eb.add_data(data)
        batch.flush()                      # returns with this round's work in flight
        for p in eb.packets[sent:]:
            if rng.random() >= 0.2:
                da.add_packet(p)
                db.add_packet(p)
        sent = len(eb.packets)
        if step == 70:
            da.set_batch(None)             # drains the batch (in flight included), then immediate
    while batch.pending:
        batch.flush()
    assert ea.packets == eb.packets
    assert da.data == db.data and da.packets == db.packets
    assert db.nb_decoded > 0
    # a second asynchronous batch; the first is deleted with its encoder's events in flight
    b2 = capi.Batch(asynchronous=True)
    ec, ed = capi.Encoder(), capi.Encoder()
    for e in (ec, ed):
        e.set_rate(2)
    ec.set_batch(b2)
    ea.set_batch(batch)
    for step in range(40):
        data = bytes([step]) * (50 + step)
        ea.add_data(data)
        ec.add_data(data)
        ed.add_data(data)
        batch.flush()
        b2.flush()
    h, batch.h = batch.h, None             # deleted with ea's events in flight: discarded
    batch.L.ntc_delete_batch(h)
    n0 = len(ea.packets)
    ea.add_data(b"after")                  # ea is unbatched again: immediate
    assert len(ea.packets) > n0
    while b2.pending:
        b2.flush()
    assert ec.packets == ed.packets
