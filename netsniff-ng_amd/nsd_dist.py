"""nsd_dist.py - multi-GPU plumbing of the dissection path.

One process per GPU.  Packets are independent, so a batch shards into
contiguous packet ranges with no data-path collective; the only exchange is
the per-protocol counter vector (NSD_NCOUNTERS x u64, 512 B), summed with one
all-reduce (RCCL over xGMI on MI355X, gloo in the CPU tests).

The reference scales capture out by processes too: N netsniff-ng processes
join one PACKET_FANOUT group (ring_rx.c:197-215, netsniff-ng.c:1379-1408) and
each dissects the packets the kernel hands its socket.  Here each rank owns
one GPU and one contiguous packet range.

bench.py runs its per-rank body through this module (rank_env, weak_shard,
reduce_counters, max_over_ranks), and `bench.py --gpus N` started without a
launcher spawns its N ranks with spawn_ranks before touching any GPU."""
import os
import socket
import subprocess
import sys

import torch


def shard_range(total, rank, world):
    """Contiguous [lo, hi) of `total` packets for `rank` (strong scaling)."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def weak_shard(per_rank, rank):
    """Weak scaling: every rank owns its own `per_rank` packets."""
    return rank * per_rank, (rank + 1) * per_rank


def rank_env():
    """(rank, world, local_rank) from a torch.distributed.run environment,
    (0, 1, 0) without one."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend, local_rank=None):
    """Join the process group of a torch.distributed.run launch: "nccl"
    (RCCL) binds this rank to GPU `local_rank`; "gloo" is the CPU test
    backend.  Returns the torch.distributed module."""
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)
    return dist


def initialized():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _grouped():
    """A process group exists (a launch of any world size, one rank included:
    its collectives then run through RCCL / gloo all the same); a plain
    single-process run has none and skips them."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def reduce_counters(counters, group=None):
    """Sum the counter vectors of all ranks in place (int64 tensor)."""
    import torch.distributed as dist
    if _grouped():
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters


def all_ranks_agree(flag, device, group=None):
    """True iff `flag` holds on every rank (MIN all-reduce of 0/1)."""
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    if _grouped():
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def barrier(group=None):
    import torch.distributed as dist
    if _grouped():
        dist.barrier(group=group)


def max_over_ranks(values, device, group=None):
    """Max of a list of floats over ranks (bench timing)."""
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if _grouped():
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(x) for x in t]


def count_devices():
    """GPUs visible, counted in a child process so the caller initialises
    no GPU runtime before it spawns its ranks (0 if the count fails)."""
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=300)
    except (subprocess.TimeoutExpired, OSError):
        return 0
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(nproc, script, argv, env=None):
    """Run `script argv` as `nproc` fresh rank processes, one per GPU, under
    torch.distributed.run on 127.0.0.1 (the caller has not touched a GPU:
    count_devices counts them in a child process), and return their exit
    code.
    The ranks' stdout is this process's: rank 0 prints the result."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script] + list(argv)
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=e).returncode
