"""ntc_gf256_gather_combine (include/netcode/gpu.h): the batching adaptor's combination over
payloads already resident on the device -- out_j[0 .. len_j) = sum_t c_t * src_t[0 .. len_t) with
sources zero-extended past their len, outputs zero-padded to 16 bytes -- against the oracle's
region multiply-add (galois_field.hh:65-92), including partial 16-byte pieces, empty terms,
lengths past 1 KiB (several waves per job) and payloads shared by several jobs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_gather_combine_matches_oracle(gpu, oracle):
    import torch
    from netcode_amd import _native
    from netcode_amd.engine import Engine, _stream
    rng = np.random.default_rng(11)
    sizes = [int(x) for x in rng.integers(0, 3000, 24)] + [0, 1, 15, 16, 17, 1024, 1025]
    pad = lambda n: (max(n, 1) + 15) // 16 * 16
    offs, pos = [], 0
    for n in sizes:
        offs.append(pos)
        pos += pad(n)
    host = np.zeros(pos, np.uint8)
    for o, n in zip(offs, sizes):
        host[o:o + n] = rng.integers(0, 256, n, dtype=np.uint8)
    jobs, terms, want = [], [], []
    out_len = [int(x) for x in rng.integers(1, 3000, 12)] + [16, 1, 2048]
    out_offs, opos = [], 0
    for L in out_len:
        out_offs.append(opos)
        opos += pad(L)
    arena = torch.from_numpy(np.concatenate([host, np.full(opos, 0xAB, np.uint8)])).to(gpu)
    base = arena.data_ptr()
    L_ = oracle.lib()
    for j, L in enumerate(out_len):
        t0 = len(terms)
        acc = np.zeros(pad(L), np.uint8)
        for i in rng.choice(len(sizes), size=int(rng.integers(0, 9)), replace=False):
            ln = int(min(sizes[i], L, rng.integers(0, sizes[i] + 1) if rng.random() < 0.3 else sizes[i]))
            c = int(rng.integers(0, 256))
            terms.append((base + offs[i], ln, c))
            seg = host[offs[i]:offs[i] + ln].copy()
            L_.or_region_muladd(oracle._p(seg), oracle._p(acc), ln, c)
        jobs.append((base + host.size + out_offs[j], 0, t0, len(terms) - t0, L, 0))
        want.append(acc)
    jd = np.array(jobs, dtype=[("out", "<u8"), ("out2", "<u8"), ("term0", "<u4"), ("nterms", "<u4"),
                               ("len", "<u4"), ("pad", "<u4")])
    td = np.array(terms or [(0, 0, 0)], dtype=[("src", "<u8"), ("len", "<u4"), ("coef", "<u4")])
    dj = torch.from_numpy(jd.view(np.uint8)).to(gpu)
    dt = torch.from_numpy(td.view(np.uint8)).to(gpu)
    L = _native.load()
    _native.check(L.ntc_gf256_gather_combine(Engine.get(gpu).handle, len(jobs), dj.data_ptr(), dt.data_ptr(),
                                             max(out_len), _stream(gpu)), "gather_combine")
    torch.cuda.synchronize(gpu)
    got = arena.cpu().numpy()[host.size:]
    for j, L in enumerate(out_len):
        o = out_offs[j]
        assert (got[o:o + pad(L)] == want[j]).all(), j
    assert (arena.cpu().numpy()[:host.size] == host).all()      # inputs untouched


def test_gather_combine_pinned_host_sources_and_second_output(gpu, oracle):
    """The adaptor's flush form: terms reading pinned host memory (this flush's new payloads) and a
    second output into pinned host memory (the result handed to callbacks)."""
    import torch
    from netcode_amd import _native
    from netcode_amd.engine import Engine, _stream
    rng = np.random.default_rng(12)
    pad = lambda n: (max(n, 1) + 15) // 16 * 16
    sizes = [1024, 1500, 17, 2100, 0, 640]
    offs, pos = [], 0
    for n in sizes:
        offs.append(pos)
        pos += pad(n)
    src = torch.zeros(pos, dtype=torch.uint8, pin_memory=True)
    data = rng.integers(0, 256, pos, dtype=np.uint8)
    for o, n in zip(offs, sizes):
        src.numpy()[o:o + n] = data[o:o + n]
    out_len = [1024, 2100, 33]
    dev_out = torch.zeros(sum(pad(L) for L in out_len), dtype=torch.uint8, device=gpu)
    host_out = torch.full((dev_out.numel(),), 0xCD, dtype=torch.uint8, pin_memory=True)
    jobs, terms, want, opos = [], [], [], 0
    L_ = oracle.lib()
    for L in out_len:
        t0, acc = len(terms), np.zeros(pad(L), np.uint8)
        for i, n in enumerate(sizes):
            ln = min(n, L)
            c = int(rng.integers(1, 256))
            terms.append((src.data_ptr() + offs[i], ln, c))
            seg = src.numpy()[offs[i]:offs[i] + ln].copy()
            L_.or_region_muladd(oracle._p(seg), oracle._p(acc), ln, c)
        jobs.append((dev_out.data_ptr() + opos, host_out.data_ptr() + opos, t0, len(terms) - t0, L, 0))
        want.append((opos, acc))
        opos += pad(L)
    jd = np.array(jobs, dtype=[("out", "<u8"), ("out2", "<u8"), ("term0", "<u4"), ("nterms", "<u4"),
                               ("len", "<u4"), ("pad", "<u4")])
    td = np.array(terms, dtype=[("src", "<u8"), ("len", "<u4"), ("coef", "<u4")])
    dj = torch.from_numpy(jd.view(np.uint8)).to(gpu)
    dt = torch.from_numpy(td.view(np.uint8)).to(gpu)
    L = _native.load()
    _native.check(L.ntc_gf256_gather_combine(Engine.get(gpu).handle, len(jobs), dj.data_ptr(), dt.data_ptr(),
                                             max(out_len), _stream(gpu)), "gather_combine")
    torch.cuda.synchronize(gpu)
    dev = dev_out.cpu().numpy()
    hst = host_out.numpy()
    for o, acc in want:
        assert (dev[o:o + acc.size] == acc).all()
        assert (hst[o:o + acc.size] == acc).all()
