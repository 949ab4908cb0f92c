"""N>1 path on CPU (gloo, world_size 2): generation sharding reproduces the single-process batch
bit for bit (ids, repairs, decode outcomes), and the bench's barrier + max-time reduction works.
The GPU ranks (bench.py --gpus N under torchrun) run the same shard code with the HIP engine and
the same gloo barrier / max-reduce on host tensors -- no collective touches the data path.  The
HIP engine itself is run per rank in tests/test_gpu_multirank.py."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, G, k, r, S):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from helpers import loss_exact_m, make_sources
    from netcode_amd.shard import generation_shard, max_over_ranks
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sid, rid = generation_shard(rank, world, G, k, r)
    src, lens = make_sources(G * world, k, S, S, seed=21)
    src, lens = src[rank * G:(rank + 1) * G], lens[rank * G:(rank + 1) * G]
    rep, rsz = O.encode_batch(src, lens, k, r, sid, rid)
    mask = loss_exact_m(G * world, k, r, seed=22)[rank * G:(rank + 1) * G]
    lost = src * mask[:, :, None]
    out, olen, st = O.decode_batch(lost, lens * mask, mask, rep, rsz, np.ones((G, r), np.uint8),
                                   sid, rid)
    dist.barrier()
    t = max_over_ranks(float(rank + 1), dist)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), rep=rep, rsz=rsz, st=st.view(np.uint8),
             out=out, tmax=np.array([t]))
    dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process(tmp_path, oracle):
    import torch.multiprocessing as mp
    from helpers import loss_exact_m, make_sources
    from netcode_amd.shard import generation_shard
    world, G, k, r, S = 2, 6, 32, 8, 64
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), G, k, r, S), nprocs=world,
                       join=True, start_method="spawn")
    sid, rid = generation_shard(0, 1, G * world, k, r)
    src, lens = make_sources(G * world, k, S, S, seed=21)
    rep, rsz = oracle.encode_batch(src, lens, k, r, sid, rid)
    mask = loss_exact_m(G * world, k, r, seed=22)
    out, olen, st = oracle.decode_batch(src * mask[:, :, None], lens * mask, mask, rep, rsz,
                                        np.ones((G * world, r), np.uint8), sid, rid)
    for rank in range(world):
        z = np.load(os.path.join(tmp_path, f"rank{rank}.npz"))
        sl = slice(rank * G, (rank + 1) * G)
        assert (z["rep"] == rep[sl]).all() and (z["rsz"] == rsz[sl]).all()
        assert (z["st"] == st[sl].view(np.uint8)).all()
        assert (z["out"] == out[sl]).all()
        assert float(z["tmax"][0]) == float(world)


def _worker_cfg4(rank, world, port, out_dir, vrank0, vworld, G, k, r, S, pick):
    """Rank `rank` plays rank vrank0 + rank of a vworld-GPU config-4 run (G generations per GPU),
    computing the generations `pick` of its shard with the shard's own id bases."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from helpers import loss_exact_m, make_sources
    from netcode_amd.shard import generation_shard, max_over_ranks
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    vr = vrank0 + rank
    sid, rid = generation_shard(vr, vworld, G, k, r)
    sid, rid = sid[pick], rid[pick]
    n = len(pick)
    src, lens = make_sources(n, k, S, S, seed=100 + vr, ragged=True)
    rep, rsz = O.encode_batch(src, lens, k, r, sid, rid)
    mask = loss_exact_m(n, k, r, seed=200 + vr)
    out, olen, st = O.decode_batch(src * mask[:, :, None], lens * mask, mask, rep, rsz,
                                   np.ones((n, r), np.uint8), sid, rid)
    t = max_over_ranks(float(vr), dist)
    np.savez(os.path.join(out_dir, f"cfg4_{vr}.npz"), sid=sid, rid=rid, rep=rep, rsz=rsz,
             st=st.view(np.uint8), out=out, olen=olen, tmax=np.array([t]))
    dist.destroy_process_group()


def test_config4_last_ranks_wrapping_ids(tmp_path, oracle):
    """Config 4 (k=128 r=32, 65536 generations over 8 GPUs), shard ids only: ranks 6 and 7 own
    the generations whose rid * sid products exceed 2^32 (galois_field.hh:143-158 wraps them).  Two
    gloo ranks play ranks 6..7 and check that generation_shard gives them the single-batch ids of
    the same generations and that the gloo max-reduce works; the repairs / outcomes compared here
    are the oracle's on both sides (no engine runs -- the HIP engine on these ids is
    test_gpu_multirank.py / test_gpu_parity.py's wrap cases)."""
    import torch.multiprocessing as mp
    from helpers import loss_exact_m, make_sources
    from netcode_amd.shard import generation_shard
    vworld, G, k, r, S = 8, 8192, 128, 32, 64
    pick = np.array([0, 1, G // 2, G - 2, G - 1])
    mp.start_processes(_worker_cfg4, args=(2, _free_port(), str(tmp_path), 6, vworld, G, k, r, S, pick),
                       nprocs=2, join=True, start_method="spawn")
    sid_all, rid_all = generation_shard(0, 1, G * vworld, k, r)
    for vr in (6, 7):
        z = np.load(os.path.join(tmp_path, f"cfg4_{vr}.npz"))
        g = vr * G + pick
        assert (z["sid"] == sid_all[g]).all() and (z["rid"] == rid_all[g]).all()
        # the products of these ids wrap uint32 (the case the shard must not "fix")
        R1, S1 = rid_all[g].astype(np.uint64) + 1, sid_all[g].astype(np.uint64) + 1
        assert ((R1 + S1) * R1 > 2**32).all()
        n = len(pick)
        src, lens = make_sources(n, k, S, S, seed=100 + vr, ragged=True)
        rep, rsz = oracle.encode_batch(src, lens, k, r, sid_all[g], rid_all[g])
        mask = loss_exact_m(n, k, r, seed=200 + vr)
        out, olen, st = oracle.decode_batch(src * mask[:, :, None], lens * mask, mask, rep, rsz,
                                            np.ones((n, r), np.uint8), sid_all[g], rid_all[g])
        assert (z["rep"] == rep).all() and (z["rsz"] == rsz).all()
        assert (z["st"] == st.view(np.uint8)).all()
        assert (z["out"] == out).all() and (z["olen"] == olen).all()
        assert float(z["tmax"][0]) == 7.0


def test_shard_ids_wrap_like_uint32():
    from netcode_amd.shard import generation_shard
    sid, rid = generation_shard(7, 8, 8192, 128, 32)
    assert sid.dtype == np.uint32 and sid[0] == 7 * 8192 * 128
    sid2, _ = generation_shard(1, 2, 4, 2**31, 1)
    assert sid2[0] == (4 * 2**31) & 0xFFFFFFFF
