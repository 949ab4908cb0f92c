"""netcode_amd -- MI355X-native GF(2^8) network-coding engine (drop-in for ahamez/netcode's
coding hot path).  The GF region multiply-accumulate, decode planning and Gauss-Jordan run in
hand-written gfx950 HIP kernels in ``libntc_gf256.so`` (C ABI: include/netcode/gpu.h)."""
from ._native import NativeError, load as load_native  # noqa: F401

__all__ = ["NativeError", "load_native", "Engine", "GaloisField", "BatchEncoder", "BatchDecoder", "DenseCode",
           "Wire"]


def __getattr__(name):
    # torch-dependent classes are imported lazily so the C-ABI checks work without torch.
    if name in ("Engine", "GaloisField", "BatchEncoder", "BatchDecoder", "status_to_numpy",
                "STATUS_DTYPE", "EncodeResult", "DenseCode", "Wire", "ReceivedBatch", "combine"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
