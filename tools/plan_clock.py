"""Per-wave timeline of decode_plan_w (experiment build exp/libntc_gf256_clk.so, -DNTC_PLAN_CLOCK):
start / after setup / after Gauss-Jordan / end stamps (wall_clock64, 100 MHz) per generation.
usage: NTC_GF256_LIB=exp/libntc_gf256_clk.so python tools/plan_clock.py [config] [G]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "k128r32s4096"
k, r, S, stride, m, Gdef = bench.CONFIGS[cfg]
G = int(sys.argv[2]) if len(sys.argv) > 2 else Gdef
dev = torch.device("cuda", 0)
w = bench.Workload(dev, G, k, r, S, stride, m, False, 0)
for _ in range(5):
    w.step()
torch.cuda.synchronize()
from netcode_amd import _native
L = _native.load()
L.ntc_dbg_plan_clock.argtypes = [C.c_void_p, C.c_uint32]
out = np.zeros(8 * G, np.uint64)
assert L.ntc_dbg_plan_clock(out.ctypes.data, 8 * G) == 0
t = out.reshape(G, 8).astype(np.int64)
t0, t1, t2, t3, st = t[:, 0], t[:, 1], t[:, 2], t[:, 3], t[:, 4]
base = t0.min()
us = lambda x: x / 100.0
res = {"config": cfg, "G": G, "span_us": us(t3.max() - base),
       "start_us_pct": [us(np.percentile(t0 - base, p)) for p in (0, 50, 90, 99, 100)]}
for name, sel in (("decoded", st == 0), ("singular", st == 3)):
    if sel.sum() == 0:
        continue
    d = t3[sel] - t0[sel]
    res[name] = {"n": int(sel.sum()), "dur_us_p50": us(np.median(d)), "dur_us_max": us(d.max()),
                 "setup_us_p50": us(np.median(t1[sel] - t0[sel])),
                 "gj_us_p50": us(np.median(t2[sel] - t1[sel])), "gj_us_max": us((t2[sel] - t1[sel]).max()),
                 "emit_us_p50": us(np.median(t3[sel] - t2[sel])),
                 "end_us_max": us(t3[sel].max() - base)}
# where the waves ran: HW_ID bits 8-15 (CU, SH, SE) + XCC id -> waves per CU and their durations
hw, xcc = t[:, 5], t[:, 6]
cu = (xcc << 8) | ((hw >> 8) & 0xFF)
_, inv, cnt = np.unique(cu, return_inverse=True, return_counts=True)
load = cnt[inv]
res["cus"] = int(len(cnt))
res["waves_per_cu_hist"] = {int(v): int((cnt == v).sum()) for v in np.unique(cnt)}
res["dur_us_p50_by_cu_waves"] = {int(v): us(float(np.median((t3 - t0)[load == v]))) for v in np.unique(load)}
res["end_us_max_by_cu_waves"] = {int(v): us(float((t3 - base)[load == v].max())) for v in np.unique(load)}
print(json.dumps(res))
