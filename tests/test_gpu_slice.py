"""Sources bit-sliced once per call (bs_preslice + gf_mac_bs<..., SL>): a combine with >= 384 rows
over whole 2 KiB spans slices its sources into an engine buffer first.  The buffer is sized on first
use, so a call captured into a graph before that use must run unsliced (no allocation during
capture) and one captured after it runs sliced -- both must equal the oracle's dense encode,
and the sliced graph must stay valid after a larger call has grown the buffer
(oracle.dense_encode: rep[j] = sum_i mat[j][i] * src[i], the reference's region multiply_add,
galois_field.hh:65-92)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_tall_combine_sliced_under_graph_capture(gpu, oracle):
    import torch
    from netcode_amd import _native
    L = _native.load()
    h = C.c_void_p()
    _native.check(L.ntc_gf256_engine_create(gpu.index or 0, C.byref(h)), "engine")   # fresh: no buffer yet
    try:
        G, k, rows, stride = 2, 40, 400, 4096
        rp = L.ntc_gf256_coef_pitch(rows)
        rng = np.random.default_rng(11)
        src = rng.integers(0, 256, (G, k, stride), dtype=np.uint8)
        mat = rng.integers(0, 256, (G, rows, k), dtype=np.uint8)
        coef = np.zeros((G, k, rp), np.uint8)
        coef[:, :, :rows] = mat.transpose(0, 2, 1)             # input-major, padded to the row tile
        ref = np.stack([oracle.dense_encode(mat[g], src[g]) for g in range(G)])
        s_t = torch.from_numpy(src).to(gpu)
        c_t = torch.from_numpy(coef).to(gpu)

        def combine(out, stream):
            _native.check(L.ntc_gf256_combine_batch(h, G, k, rows, stride, s_t.data_ptr(), c_t.data_ptr(),
                                                    out.data_ptr(), stream), "combine")

        def capture():
            out = torch.full((G, rows, stride), 0xA5, dtype=torch.uint8, device=gpu)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                combine(out, torch.cuda.current_stream(gpu).cuda_stream)
            return graph, out

        def replay(graph, out):
            out.fill_(0xA5)
            graph.replay()
            torch.cuda.synchronize(gpu)
            return out.cpu().numpy()

        assert (replay(*capture()) == ref).all()               # before any sizing: unsliced
        out = torch.empty((G, rows, stride), dtype=torch.uint8, device=gpu)
        _native.check(L.ntc_gf256_timing_log(h, 8), "timing log")
        combine(out, torch.cuda.current_stream(gpu).cuda_stream)   # sizes the sliced copy
        n = C.c_uint32()
        kinds, ms = (C.c_uint32 * 8)(), (C.c_float * 8)()
        _native.check(L.ntc_gf256_timing_read(h, 8, C.byref(n), C.addressof(kinds), C.addressof(ms)),
                      "timing read")
        _native.check(L.ntc_gf256_timing_log(h, 0), "timing log off")
        assert list(kinds[:n.value]) == [8, 1]                 # NTC_GF256_K_SLICE, then the MAC
        torch.cuda.synchronize(gpu)
        assert (out.cpu().numpy() == ref).all()
        sliced = capture()
        assert (replay(*sliced) == ref).all()                  # buffer present: sliced in the graph
        # a later, larger call grows the sliced copy: the old one must outlive the graph that
        # addresses it (retired, not freed, once the engine has seen a capture)
        big = torch.zeros((G, 2 * k, stride), dtype=torch.uint8, device=gpu)
        big_c = torch.zeros((G, 2 * k, rp), dtype=torch.uint8, device=gpu)
        big_o = torch.empty((G, rows, stride), dtype=torch.uint8, device=gpu)
        _native.check(L.ntc_gf256_combine_batch(h, G, 2 * k, rows, stride, big.data_ptr(), big_c.data_ptr(),
                                                big_o.data_ptr(), torch.cuda.current_stream(gpu).cuda_stream),
                      "larger combine")
        torch.cuda.synchronize(gpu)
        assert not big_o.any()
        assert (replay(*sliced) == ref).all()
        # once the graphs are gone the retired buffers can be freed; the engine keeps working
        del sliced
        torch.cuda.synchronize(gpu)
        _native.check(L.ntc_gf256_release_retired(h), "release retired")
        out.fill_(0xA5)
        combine(out, torch.cuda.current_stream(gpu).cuda_stream)
        torch.cuda.synchronize(gpu)
        assert (out.cpu().numpy() == ref).all()
    finally:
        torch.cuda.synchronize(gpu)
        L.ntc_gf256_engine_destroy(h)
