"""Regenerate tests/golden/*.npz from the pinned CPU oracle (oracle/ntc_oracle.c).

The oracle itself is pinned by tests/golden/kat.json (SURVEY §8(c) KATs + §6 end_to_end
counters of the reference build); these vectors freeze its decode outcomes (including singular
generations) so the GPU tests compare against committed data as well as the live oracle.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
from helpers import loss_iid, make_sources  # noqa: E402

CASES = {
    # config 1 generation form: k=16 r=4 1 KiB, i.i.d. 25 % loss on sources and repairs
    "gen_k16_r4_loss25": dict(G=400, k=16, r=4, S=32, stride=32, seed=11, p=0.25, ragged=False),
    # config 2 shape at reduced G, ragged sizes
    "gen_k32_r8_ragged": dict(G=48, k=32, r=8, S=200, stride=208, seed=12, p=0.2, ragged=True),
}


def make(name, G, k, r, S, stride, seed, p, ragged):
    src, lens = make_sources(G, k, S, stride, seed, ragged)
    sid = (np.arange(G, dtype=np.uint64) * k + 7).astype(np.uint32)
    rid = (np.arange(G, dtype=np.uint64) * r + 3).astype(np.uint32)
    rep, rsz = O.encode_batch(src, lens, k, r, sid, rid)
    smask = loss_iid((G, k), p, seed + 1)
    rmask = loss_iid((G, r), p, seed + 2)
    lost = src.copy()
    lost[smask == 0] = 0
    llen = lens.copy()
    llen[smask == 0] = 0
    out, olen, st = O.decode_batch(lost, llen, smask, rep, rsz, rmask, sid, rid)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), src=src, src_len=lens, sid_base=sid,
                        rid_base=rid, rep=rep, rep_size=rsz, src_mask=smask, rep_mask=rmask,
                        out=out, out_len=olen, status=st.view(np.uint8).reshape(G, -1))
    print(name, "states:", np.bincount(st["state"], minlength=4).tolist())


if __name__ == "__main__":
    O.build()
    for n, c in CASES.items():
        make(n, **c)
