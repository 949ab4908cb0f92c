"""CPU tests of the per-packet netcode C ABI library (libntc.so): it loads, exports every
function include/netcode/c/*.h declares, its data/packet buffers behave like the reference's
(c/data.cc, c/packet.cc), and without a HIP device encoder/decoder creation fails loudly."""
import ctypes as C

import pytest


def test_exports_all_declared_symbols(native_built):
    from netcode_amd import capi
    L = capi.load()
    names = capi.header_symbols()
    assert len(names) >= 28 + 2
    for n in names:
        assert hasattr(L, n), n


def test_reference_abi_names_present(native_built):
    # the 28 functions of the reference's netcode/c ABI
    ref = """ntc_new_data ntc_new_data_from ntc_delete_data ntc_data_buffer ntc_data_get_size
    ntc_data_resize ntc_new_packet ntc_new_packet_from ntc_delete_packet ntc_packet_buffer
    ntc_packet_get_size ntc_packet_resize ntc_new_encoder ntc_delete_encoder ntc_encoder_add_data
    ntc_encoder_add_packet ntc_encoder_generate_repair ntc_encoder_window ntc_encoder_set_code_type
    ntc_encoder_set_rate ntc_encoder_set_window_size ntc_encoder_set_adaptive ntc_new_decoder
    ntc_delete_decoder ntc_decoder_add_packet ntc_decoder_generate_ack ntc_decoder_set_ack_period
    ntc_decoder_set_ack_nb_packets""".split()
    assert len(ref) == 28
    from netcode_amd import capi
    assert set(ref) <= set(capi.header_symbols())


def test_data_and_packet_buffers(native_built):
    from netcode_amd import capi
    L = capi.load()
    d = L.ntc_new_data_from(b"abc", 3)
    assert L.ntc_data_get_size(d) == 3 and C.string_at(L.ntc_data_buffer(d), 3) == b"abc"
    assert L.ntc_data_buffer(d) % 16 == 0
    err = capi.Error(0, None)
    L.ntc_data_resize(d, 1024, C.byref(err))
    assert err.type == 0 and L.ntc_data_get_size(d) == 1024
    L.ntc_delete_data(d)
    p = L.ntc_new_packet(1024)
    assert L.ntc_packet_get_size(p) == 1024
    assert (L.ntc_packet_buffer(p) + 7) % 16 == 0      # symbol after the 7-byte header is aligned
    L.ntc_packet_resize(p, 11, C.byref(err))
    assert L.ntc_packet_get_size(p) == 11
    L.ntc_delete_packet(p)


def test_no_device_means_no_encoder(native_built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from netcode_amd import capi
    L = capi.load()
    c = capi._Collector()
    assert not L.ntc_new_encoder(8, c.handler)
    assert not L.ntc_new_decoder(8, 0, c.handler, capi.DataHandler(None, capi.READ(lambda *a: None)))
