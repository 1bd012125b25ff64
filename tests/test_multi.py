"""world_size-2 gloo test of the multi-GPU design on CPU: contiguous shards
cover the batch exactly once, and all-reducing the per-rank counter vectors
gives the counters of the whole batch (counters computed per shard by the CPU
oracle standing in for each rank's device)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import nsd_dist
import nsd_testlib as T


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, cfg, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = nsd_dist.shard_range(total, rank, world)
    frames, desc = T.make_batch(cfg, hi - lo, lo=lo)
    _, _, cnt, _ = T.oracle_records(frames, desc)
    c = torch.from_numpy(cnt.view(np.int64).copy())
    nsd_dist.reduce_counters(c)
    m = nsd_dist.max_over_ranks([float(rank)], "cpu")
    if rank == 0:
        np.save(out, c.numpy())
        assert m == [float(world - 1)]
    dist.destroy_process_group()


def test_sharded_counters_allreduce(tmp_path):
    world, total = 2, 40000
    for cfg in (T.SYN_IMIX, T.SYN_IPV6X):
        out = str(tmp_path / f"c{cfg}.npy")
        mp.spawn(_worker, args=(world, _free_port(), total, cfg, out), nprocs=world, join=True)
        got = np.load(out).view(np.uint64)
        frames, desc = T.make_batch(cfg, total)
        _, _, want, _ = T.oracle_records(frames, desc)
        assert np.array_equal(got, want)
        assert int(got[32]) == total


def test_shards_partition_exactly():
    for total in (0, 1, 7, 1000, 2 ** 24 + 3):
        for world in (1, 2, 3, 8):
            rngs = [nsd_dist.shard_range(total, r, world) for r in range(world)]
            assert rngs[0][0] == 0 and rngs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rngs, rngs[1:]))
    assert nsd_dist.weak_shard(16, 3) == (48, 64)
