"""Timeline of the lookahead inversion launches (experiment build with -DNTC_DENSE_CLOCK):
per launch, the panel block's stamps (start, tables + T staged, owner rows derived, owner phase
done, end) and the update blocks' first start / last end, in us (wall_clock64, 100 MHz).
usage: NTC_GF256_LIB=exp/libntc_gf256_dnclk.so python tools/dense_clock.py [--n 1024]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netcode_amd import _native  # noqa: E402
from netcode_amd.engine import DenseCode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1024)
a = ap.parse_args()
g = torch.Generator().manual_seed(5)
mat = torch.randint(0, 256, (1, a.n, a.n), dtype=torch.uint8, generator=g).cuda()
dc = DenseCode(0)
for _ in range(3):
    dc.invert(mat)
torch.cuda.synchronize()
L = _native.load()
L.ntc_dbg_dense_clock.argtypes = [C.c_void_p, C.c_uint32, C.c_int]
assert L.ntc_dbg_dense_clock(None, 0, 1) == 0
dc.invert(mat)
torch.cuda.synchronize()
out = np.zeros(64 * 8, np.uint64)
assert L.ntc_dbg_dense_clock(out.ctypes.data, 64 * 8, 0) == 0
t = out.reshape(64, 8).astype(np.int64)
rows = [i for i in range(64) if t[i, 0] and t[i, 4]]
us = lambda x: round(float(x) / 100.0, 2)
per = []
for i in rows:
    t0 = t[i, 0]
    per.append({"panel": i, "stage": us(t[i, 1] - t0), "derive": us(t[i, 2] - t[i, 1]),
                "owner": us(t[i, 3] - t[i, 2]), "tail": us(t[i, 4] - t[i, 3]), "panel_total": us(t[i, 4] - t0),
                "upd_start": us(t[i, 6] - t0), "upd_end": us(t[i, 7] - t0),
                "gap_to_next": us(t[i + 1, 0] - max(t[i, 4], t[i, 7])) if i + 1 in rows else None})
med = {k: float(np.median([p[k] for p in per if p[k] is not None])) for k in per[0] if k != "panel"}
print(json.dumps({"n": a.n, "launches": len(per), "median": med, "first": per[:3], "last": per[-2:]}))
