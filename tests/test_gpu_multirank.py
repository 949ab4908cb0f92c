"""GPU: the N > 1 path with the HIP engine doing the work on every rank.  Two processes (gloo for
the barrier / max-reduce, both on the box's one GPU) each encode and decode their generation
shard (netcode_amd.shard.generation_shard id bases) through BatchEncoder / BatchDecoder; the
union is bit-identical to the oracle over the whole batch.  And bench.py itself under torchrun
with two ranks (its default gloo rank sync) prints one line with n_gpus = 2 and a verified round
trip -- the driver's multi-GPU launch shape, minus RCCL."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, G, k, r, S):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from helpers import loss_exact_m, make_sources
    from netcode_amd import BatchDecoder, BatchEncoder, status_to_numpy
    from netcode_amd.shard import generation_shard, max_over_ranks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    sid, rid = generation_shard(rank, world, G, k, r)
    src, lens = make_sources(G * world, k, S, S, seed=31)
    src, lens = src[rank * G:(rank + 1) * G], lens[rank * G:(rank + 1) * G]
    mask = loss_exact_m(G * world, k, r, seed=32)[rank * G:(rank + 1) * G]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_sid, d_rid = t(sid.view(np.int32)), t(rid.view(np.int32))
    res = BatchEncoder(k, r, dev)(t(src), t(lens.view(np.int16)), d_sid, d_rid)
    rx = t(src * mask[:, :, None])
    rxl = t((lens * mask).view(np.int16))
    st = BatchDecoder(k, r, dev)(rx, rxl, t(mask), res.repairs, res.encoded_size,
                                 torch.ones((G, r), dtype=torch.uint8, device=dev), d_sid, d_rid)
    torch.cuda.synchronize(dev)
    dist.barrier()
    tmax = max_over_ranks(float(rank + 1), dist, dev)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), rep=res.repairs.cpu().numpy(),
             rsz=res.encoded_size.cpu().numpy().view(np.uint16), out=rx.cpu().numpy(),
             olen=rxl.cpu().numpy().view(np.uint16), st=status_to_numpy(st).view(np.uint8),
             tmax=np.array([tmax]))
    dist.destroy_process_group()


def test_two_gpu_ranks_match_single_batch_oracle(tmp_path, oracle):
    import torch.multiprocessing as mp
    from helpers import loss_exact_m, make_sources
    from netcode_amd.shard import generation_shard
    world, G, k, r, S = 2, 24, 32, 8, 1024
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), G, k, r, S), nprocs=world,
                       join=True, start_method="spawn")
    sid, rid = generation_shard(0, 1, G * world, k, r)
    src, lens = make_sources(G * world, k, S, S, seed=31)
    rep, rsz = oracle.encode_batch(src, lens, k, r, sid, rid)
    mask = loss_exact_m(G * world, k, r, seed=32)
    out, olen, st = oracle.decode_batch(src * mask[:, :, None], lens * mask, mask, rep, rsz,
                                        np.ones((G * world, r), np.uint8), sid, rid)
    for rank in range(world):
        z = np.load(os.path.join(tmp_path, f"rank{rank}.npz"))
        sl = slice(rank * G, (rank + 1) * G)
        assert (z["rep"] == rep[sl]).all()
        assert (z["rsz"] == rsz[sl]).all()
        assert (z["st"].reshape(-1) == st[sl].view(np.uint8).reshape(-1)).all()
        assert (z["out"] == out[sl]).all()
        assert (z["olen"] == olen[sl]).all()
        assert float(z["tmax"][0]) == world


def _ndev():
    import torch
    return torch.cuda.device_count()


def test_bench_under_torchrun_two_ranks(tmp_path):
    env = {k_: v for k_, v in os.environ.items() if k_ != "NTC_BENCH_BACKEND"}   # the default: gloo
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--G", "256", "--no-cpu-baseline", "--no-host-rate"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]           # rank 0 prints the only line
    d = json.loads(lines[0])
    # both ranks share this box's device: the line counts distinct devices and ranks apart
    assert d["ranks"] == 2 and d["n_gpus"] == min(2, _ndev()) and d["value"] > 0
    assert d["verified"]["bit_exact_round_trip"]
    assert d["rank_sync"] == "gloo"                    # no RCCL for the barrier / max
    assert d["config"]["generations_per_gpu"] == 256


def _worker_cfg4(rank, world, port, out_dir, vrank0, vworld, Gshard, k, r, S, pick):
    """Rank `rank` plays rank vrank0 + rank of config 4's vworld-GPU run: the HIP engine encodes
    and decodes the generations `pick` of its shard with that shard's (uint32-wrapping) ids."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from helpers import loss_exact_m, make_sources
    from netcode_amd import BatchDecoder, BatchEncoder, status_to_numpy
    from netcode_amd.shard import generation_shard, max_over_ranks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    vr = vrank0 + rank
    sid, rid = generation_shard(vr, vworld, Gshard, k, r)
    sid, rid = sid[pick], rid[pick]
    n = len(pick)
    src, lens = make_sources(n, k, S, S, seed=100 + vr, ragged=True)
    mask = loss_exact_m(n, k, r, seed=200 + vr)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_sid, d_rid = t(sid.view(np.int32)), t(rid.view(np.int32))
    res = BatchEncoder(k, r, dev)(t(src), t(lens.view(np.int16)), d_sid, d_rid)
    rx = t(src * mask[:, :, None])
    rxl = t((lens * mask).view(np.int16))
    st = BatchDecoder(k, r, dev)(rx, rxl, t(mask), res.repairs, res.encoded_size,
                                 torch.ones((n, r), dtype=torch.uint8, device=dev), d_sid, d_rid)
    torch.cuda.synchronize(dev)
    tmax = max_over_ranks(float(vr), dist, dev)
    np.savez(os.path.join(out_dir, f"cfg4_{vr}.npz"), rep=res.repairs.cpu().numpy(),
             rsz=res.encoded_size.cpu().numpy().view(np.uint16), out=rx.cpu().numpy(),
             olen=rxl.cpu().numpy().view(np.uint16), st=status_to_numpy(st).view(np.uint8),
             tmax=np.array([tmax]))
    dist.destroy_process_group()


def test_config4_ranks_6_7_on_the_engine(tmp_path, oracle):
    """Config 4 (k=128 r=32, 65536 generations over 8 GPUs): two processes play ranks 6 and 7,
    whose rid * sid products exceed 2^32 (galois_field.hh:143-158 wraps them), and run their
    shards' generations through the HIP engine; repairs, sizes, outcomes and recovered payloads
    equal the oracle's over the single-batch ids of the same generations."""
    import torch.multiprocessing as mp
    from helpers import loss_exact_m, make_sources
    from netcode_amd.shard import generation_shard
    vworld, Gs, k, r, S = 8, 8192, 128, 32, 1504
    pick = np.array([0, 1, 2, Gs // 2, Gs - 3, Gs - 2, Gs - 1])
    mp.start_processes(_worker_cfg4, args=(2, _free_port(), str(tmp_path), 6, vworld, Gs, k, r, S, pick),
                       nprocs=2, join=True, start_method="spawn")
    sid_all, rid_all = generation_shard(0, 1, Gs * vworld, k, r)
    for vr in (6, 7):
        z = np.load(os.path.join(tmp_path, f"cfg4_{vr}.npz"))
        g = vr * Gs + pick
        R1, S1 = rid_all[g].astype(np.uint64) + 1, sid_all[g].astype(np.uint64) + 1
        assert ((R1 + S1) * R1 > 2**32).all()       # the wrapping products
        n = len(pick)
        src, lens = make_sources(n, k, S, S, seed=100 + vr, ragged=True)
        rep, rsz = oracle.encode_batch(src, lens, k, r, sid_all[g], rid_all[g])
        mask = loss_exact_m(n, k, r, seed=200 + vr)
        out, olen, st = oracle.decode_batch(src * mask[:, :, None], lens * mask, mask, rep, rsz,
                                            np.ones((n, r), np.uint8), sid_all[g], rid_all[g])
        assert (z["rep"] == rep).all() and (z["rsz"] == rsz).all()
        assert (z["st"].reshape(-1) == st.view(np.uint8).reshape(-1)).all()
        assert (z["out"] == out).all() and (z["olen"] == olen).all()
        assert float(z["tmax"][0]) == 7.0
