"""GPU parity of GF(2^w), w in {4, 8, 16, 32}: the device region and batched
combine kernels (ntc_gf_region_multiply / ntc_gf_combine_batch) against the oracle, and the
per-packet C ABI (libntc.so) built with galois_field_size 4 / 16 / 32 against the oracle's
streaming restatement, packet for packet and delivery for delivery."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
WS = (4, 8, 16, 32)


def cmax(w):
    return (1 << w) - 1 if w < 32 else 0xFFFFFFFF


@pytest.mark.parametrize("w", WS)
def test_region_multiply(gpu, oracle, w):
    import torch
    from netcode_amd import GaloisField
    gf = GaloisField(w, gpu)
    rng = np.random.default_rng(w)
    for n in (1, 3, 4, 17, 1024, 1501, 65536):
        src = rng.integers(0, 256, n, dtype=np.uint8)
        dst = rng.integers(0, 256, n, dtype=np.uint8)
        for c in (0, 1, 2, int(rng.integers(1, cmax(w), dtype=np.uint64)), cmax(w)):
            for add in (False, True):
                s_t = torch.from_numpy(src).to(gpu)
                d_t = torch.from_numpy(dst.copy()).to(gpu)
                (gf.multiply_add if add else gf.multiply)(s_t, d_t, n, c)
                torch.cuda.synchronize()
                want = oracle.fw_region(w, src, dst, c, add)
                assert (d_t.cpu().numpy() == want).all(), (n, c, add)


@pytest.mark.parametrize("w", WS)
# row groups of 8 / 4 / 2 / 1 per wave, 256 B - 1 KiB column spans (ragged last span), all-zero
# sources; both kernel forms: the table lookups (default) and the masked shift-and-add
@pytest.mark.parametrize("G,k,rows,stride", [(3, 5, 2, 64), (2, 17, 4, 1504), (1, 1, 1, 16), (2, 6, 9, 2064),
                                             (1, 3, 8, 1024), (4, 33, 3, 48), (1, 4, 19, 1040),
                                             (2, 7, 16, 272), (1, 9, 5, 528)])
@pytest.mark.parametrize("form", ["fr", "mask"])
def test_combine_batch(gpu, oracle, monkeypatch, w, G, k, rows, stride, form):
    import torch
    from netcode_amd import combine
    monkeypatch.setenv("NTC_GFW_KERNEL", form)
    rng = np.random.default_rng(G * 100 + k + w)
    x = rng.integers(0, 256, (G, k, stride), dtype=np.uint8)
    cf = rng.integers(0, cmax(w), (G, k, rows), dtype=np.uint64, endpoint=True).astype(np.uint32)
    cf[0, 0, 0] = 0
    if k > 2:
        cf[-1, 1, :] = 0                          # a source no row uses (skipped by the wave)
    out = combine(w, torch.from_numpy(x).to(gpu), torch.from_numpy(cf.view(np.int32)).to(gpu))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for g in range(G):
        for j in range(rows):
            acc = np.zeros(stride, np.uint8)
            for i in range(k):
                acc = oracle.fw_region(w, x[g, i], acc, int(cf[g, i, j]), True)
            assert (got[g, j] == acc).all(), (g, j)


@pytest.fixture(scope="module")
def capi(gpu):
    from netcode_amd import capi as c
    c.load()
    return c


@pytest.mark.parametrize("w", (4, 16, 32))
@pytest.mark.parametrize("systematic,rate,window", [(True, 3, 12), (False, 4, 6)])
def test_capi_encoder_packets(capi, oracle, w, systematic, rate, window):
    rng = np.random.default_rng(w + rate)
    a, b = capi.Encoder(w), oracle.Encoder(galois_field_size=w)
    for e in (a, b):
        e.set_rate(rate)
        e.set_code_type(systematic)
        e.set_window_size(window)
    for i in range(40):
        data = rng.integers(0, 256, 4 * int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
        a.add_data(data)
        b.add_data(data)
        if i % 9 == 8:
            a.generate_repair()
            b.generate_repair()
    assert a.packets == b.packets


@pytest.mark.parametrize("w", (4, 16, 32))
@pytest.mark.parametrize("in_order,p_loss", [(True, 0.15), (False, 0.3)])
def test_capi_decoder_stream(capi, oracle, w, in_order, p_loss):
    rng = np.random.default_rng(10 * w + int(100 * p_loss))
    enc = oracle.Encoder(galois_field_size=w)
    enc.set_rate(3)
    enc.set_window_size(16)
    sent = []
    for i in range(150):
        d = rng.integers(0, 256, 4 * int(rng.integers(1, 200)), dtype=np.uint8).tobytes()
        sent.append(d)
        enc.add_data(d)
    pkts = [p for p in enc.packets if rng.random() >= p_loss]
    a, b = capi.Decoder(w, in_order=in_order), oracle.Decoder(in_order=in_order, galois_field_size=w)
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
    if p_loss < 0.2:
        assert b.nb_decoded > 0
    if w != 32:     # w = 32 sizes go through galois_field.hh:118's truncated product
        got = dict(b.data)
        assert all(got[i] == sent[i] for i in got)
