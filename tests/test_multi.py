"""world_size-2 gloo tests of the multi-GPU path on CPU.

test_bench_rank_body runs bench.py's own per-rank body (bench.measure_rank:
weak shards from nsd_dist.weak_shard, barrier + timed steps, the counter
all-reduce nsd_dist.reduce_counters inside the timed region, times maxed by
nsd_dist.max_over_ranks, the counter check) with each rank's shard walked by
the product's host walk (nsd.walk_cpu -> nsd_walk_packet_cpu) in place of
the kernel; the summed counters must equal the CPU oracle's over the whole
job, times the step count.  test_spawn_refuses_missing_gpus checks that
`bench.py --gpus N` without a launcher fails non-zero when fewer than N GPUs
are visible (here: none), before touching any."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import nsd_dist
import nsd_testlib as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, key, per_rank, steps, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"], os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"] = str(rank), str(world), str(rank)
    sys.path.insert(0, ROOT)
    import bench
    nsd_dist.init("gloo")
    r, w, _ = nsd_dist.rank_env()
    args = bench.parse_args(["--gpus", str(w), "--config", key, "--packets", str(per_rank), "--steps", str(steps),
                             "--warmup", "1"])
    _, m = bench.measure_rank(args, r, w, "cpu", engine="host")
    if r == 0:
        np.save(out, np.concatenate([m["counters"].view(np.int64), [m["total_pkts"]]]))
    dist.destroy_process_group()


def test_bench_rank_body(tmp_path):
    world, per_rank, steps = 2, 6000, 2
    for key, cfg in (("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)):
        out = str(tmp_path / f"{key}.npy")
        mp.spawn(_worker, args=(world, nsd_dist.free_port(), key, per_rank, steps, out), nprocs=world, join=True)
        res = np.load(out)
        got, total = res[:-1].view(np.uint64), int(res[-1])
        assert total == world * per_rank
        frames, desc = T.make_batch(cfg, world * per_rank)          # both ranks' shards
        _, _, want, _ = T.oracle_records(frames, desc)
        assert np.array_equal(got, want * np.uint64(steps))
        assert int(got[32]) == world * per_rank * steps


def _run_worker(rank, world, port, per_rank, steps, out):
    """One rank of bench.run (the N-rank output path of `bench.py --gpus N`)
    with the host engine: the headline C2 and the C3 / C4 legs, each walked
    by measure_rank and all-reduced; rank 0 saves the JSON line."""
    import json
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"], os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"] = str(rank), str(world), str(rank)
    sys.path.insert(0, ROOT)
    import bench
    nsd_dist.init("gloo")
    r, w, _ = nsd_dist.rank_env()
    args = bench.parse_args(["--gpus", str(w), "--packets", str(per_rank), "--steps", str(steps), "--warmup", "1"])
    line = bench.run(args, r, w, "cpu", engine="host")
    assert (line is None) == (r != 0)
    if r == 0:
        with open(out, "w") as f:
            json.dump(line, f)
    dist.destroy_process_group()


def test_bench_line_n_ranks(tmp_path):
    """`bench.py --gpus 2`'s line carries both north_star workloads (64 B C2
    headline, IMIX leg: C5's layout at 8 ranks) and C4, each measured at
    this N with its counters all-reduced over the ranks; the counters equal
    the oracle's over both ranks' shards x the steps."""
    import json
    import bench
    import nsd
    world, per_rank, steps = 2, 4000, 2
    out = str(tmp_path / "line.json")
    mp.spawn(_run_worker, args=(world, nsd_dist.free_port(), per_rank, steps, out), nprocs=world, join=True)
    with open(out) as f:
        line = json.load(f)
    assert line["n_gpus"] == world and line["scaling"] == "weak" and line["config"]["parallelism"] == "dp2"
    assert set(line["legs"]) == {"imix", "ipv6x"}
    assert "IMIX" in line["legs"]["imix"]["workload"] and "sharded across 2 GPUs" in line["legs"]["imix"]["workload"]
    frames, desc = T.make_batch(T.SYN_UDP64, world * per_rank)
    _, _, want, _ = T.oracle_records(frames, desc)
    assert line["counters_total"] == world * per_rank * steps
    for key, cfg in (("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)):
        leg = line["legs"][key]
        assert leg["packets"] == world * per_rank and leg["value"] > 0
        frames, desc = T.make_batch(cfg, world * per_rank)
        _, _, want, _ = T.oracle_records(frames, desc)
        assert leg["counters"] == nsd.unpack_counters(want * np.uint64(steps)), key
    assert bench.golden_counters("imix", 1 << 24, 8) is not None   # the C5 shards are in the table


def test_bench_cli_n_ranks():
    """The launch path the driver's N-GPU run takes, end to end on CPU:
    `python bench.py --gpus 2` with no launcher -> nsd_dist.spawn_ranks ->
    torch.distributed.run -> main() in each rank -> nsd_dist.init -> run()
    (the hidden --engine host switch: gloo and the product's host walk in
    place of RCCL and the kernels).  Rank 0's line: n_gpus 2, the legs, and
    the all-reduced counters equal the oracle's over both ranks' shards x
    the steps."""
    import json
    import nsd
    world, per_rank, steps = 2, 3000, 2
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--engine", "host",
                        "--packets", str(per_rank), "--steps", str(steps), "--warmup", "1", "--no-pmc"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout.decode()[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["config"]["parallelism"] == "dp2" and line["scaling"] == "weak"
    assert line["counters_total"] == world * per_rank * steps and line["setup_s"] >= 0
    assert line["bench_wall_s"] > 0
    assert set(line["legs"]) == {"imix", "ipv6x"}
    for key, cfg in (("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)):
        leg = line["legs"][key]
        assert leg["packets"] == world * per_rank and leg["schedule"] == "host walk"
        frames, desc = T.make_batch(cfg, world * per_rank)
        _, _, want, _ = T.oracle_records(frames, desc)
        assert leg["counters"] == nsd.unpack_counters(want * np.uint64(steps)), key


def _dev_worker(rank, world, port, key, per_rank, steps, out):
    """One rank of the device branch: both ranks on cuda:0 (one GPU box),
    gloo over CUDA tensors (RCCL refuses two ranks on one device)."""
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"], os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"] = str(rank), str(world), str(rank)
    sys.path.insert(0, ROOT)
    import bench
    torch.cuda.set_device(0)
    nsd_dist.init("gloo")
    r, w, _ = nsd_dist.rank_env()
    args = bench.parse_args(["--gpus", str(w), "--config", key, "--packets", str(per_rank), "--steps", str(steps),
                             "--warmup", "1"])
    b, m = bench.measure_rank(args, r, w, torch.device("cuda", 0), engine="device")
    assert b.counters.is_cuda and m["accumulate"]
    if r == 0:
        np.save(out, np.concatenate([m["counters"].view(np.int64), [m["total_pkts"]], [m["kern_ms"] > 0]]))
    b.free()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("key,cfg", [("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)])
def test_bench_rank_body_device(tmp_path, key, cfg):
    """bench.measure_rank's device branch with world size 2: each rank's
    shard resident on the GPU and walked by the kernels, all_ranks_agree /
    reduce_counters / max_over_ranks on device tensors (the reference scales
    out by processes too: PACKET_FANOUT, ring_rx.c:197-215).  The summed
    counters equal the oracle's over both shards x the steps."""
    world, per_rank, steps = 2, 1 << 16, 3
    out = str(tmp_path / f"{key}.npy")
    mp.spawn(_dev_worker, args=(world, nsd_dist.free_port(), key, per_rank, steps, out), nprocs=world, join=True)
    res = np.load(out)
    got, total, timed = res[:-2].view(np.uint64), int(res[-2]), int(res[-1])
    assert total == world * per_rank and timed == 1
    frames, desc = T.make_batch(cfg, world * per_rank)
    _, _, want, _ = T.oracle_records(frames, desc)
    assert np.array_equal(got, want * np.uint64(steps))


def test_spawn_refuses_missing_gpus():
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert r.returncode == 2 and b"GPU(s) visible" in r.stderr


def test_shards_partition_exactly():
    for total in (0, 1, 7, 1000, 2 ** 24 + 3):
        for world in (1, 2, 3, 8):
            rngs = [nsd_dist.shard_range(total, r, world) for r in range(world)]
            assert rngs[0][0] == 0 and rngs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rngs, rngs[1:]))
    assert nsd_dist.weak_shard(16, 3) == (48, 64)


def _nccl_worker(rank, world, port, per_rank, steps, out):
    """bench.run under an RCCL process group of one rank on cuda:0 (a
    one-GPU box cannot hold two RCCL ranks): nsd_dist.init("nccl") binds
    the device, and the counter all-reduce, the agreement MIN, the barrier
    and the MAX of the times go through RCCL on device tensors."""
    import json
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"], os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"] = str(rank), str(world), str(rank)
    sys.path.insert(0, ROOT)
    import bench
    nsd_dist.init("nccl", 0)
    calls = []
    real = dist.all_reduce

    def counted(t, *a, **k):
        calls.append(t.device.type)
        return real(t, *a, **k)
    dist.all_reduce = counted
    try:
        args = bench.parse_args(["--gpus", "1", "--packets", str(per_rank), "--steps", str(steps), "--warmup", "1",
                                 "--no-cpu", "--no-e2e", "--no-replay", "--no-bpf", "--no-pmc"])
        line = bench.run(args, 0, 1, torch.device("cuda", 0), "device")
    finally:
        dist.all_reduce = real
    line["_backend"] = dist.get_backend()
    line["_allreduce_devices"] = calls
    with open(out, "w") as f:
        json.dump(line, f)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_bench_run_rccl_one_rank(tmp_path):
    """The N-rank path of bench.py with the backend the driver's 8-GPU run
    uses (nccl = RCCL), at the one rank a one-GPU box allows: the line's
    headline and legs come out of RCCL collectives on GPU tensors, and the
    all-reduced counters equal the oracle's over the shard x the steps."""
    import json
    import nsd
    per_rank, steps = 1 << 16, 3
    out = str(tmp_path / "line.json")
    mp.spawn(_nccl_worker, args=(1, nsd_dist.free_port(), per_rank, steps, out), nprocs=1, join=True)
    with open(out) as f:
        line = json.load(f)
    assert line["_backend"] == "nccl"
    assert line["_allreduce_devices"] and set(line["_allreduce_devices"]) == {"cuda"}
    assert line["n_gpus"] == 1 and line["counters_total"] == per_rank * steps
    assert set(line["legs"]) == {"imix", "ipv6x"}
    for key, cfg in (("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)):
        leg = line["legs"][key]
        frames, desc = T.make_batch(cfg, per_rank)
        _, _, want, _ = T.oracle_records(frames, desc)
        assert leg["counters"] == nsd.unpack_counters(want * np.uint64(steps)), key
