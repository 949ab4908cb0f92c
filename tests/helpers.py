"""Seeded synthetic generations shared by the parity tests and the bench."""
from __future__ import annotations

import numpy as np


def make_sources(G: int, k: int, S: int, stride: int, seed: int, ragged: bool = False):
    """src [G][k][stride] uint8 zero-padded after src_len; src_len [G][k] uint16."""
    rng = np.random.default_rng(seed)
    if ragged:
        lens = rng.integers(1, S + 1, size=(G, k), dtype=np.int64).astype(np.uint16)
    else:
        lens = np.full((G, k), S, np.uint16)
    src = rng.integers(0, 256, size=(G, k, stride), dtype=np.uint8)
    col = np.arange(stride)[None, None, :]
    src[col >= lens[:, :, None]] = 0
    return src, lens


def loss_exact_m(G: int, k: int, m: int, seed: int):
    """src_mask with exactly m lost sources per generation (uniform without replacement)."""
    rng = np.random.default_rng(seed)
    mask = np.ones((G, k), np.uint8)
    for g in range(G):
        mask[g, rng.choice(k, size=m, replace=False)] = 0
    return mask


def loss_mixed_m(G: int, k: int, m_max: int, seed: int):
    rng = np.random.default_rng(seed)
    mask = np.ones((G, k), np.uint8)
    for g in range(G):
        m = int(rng.integers(0, m_max + 1))
        if m:
            mask[g, rng.choice(k, size=m, replace=False)] = 0
    return mask


def loss_iid(shape, p_loss: float, seed: int):
    rng = np.random.default_rng(seed)
    return (rng.random(shape) >= p_loss).astype(np.uint8)
