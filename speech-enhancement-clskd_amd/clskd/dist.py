"""One-process-per-GPU data parallelism for the CLSKD step (SURVEY.md §8 e).

The fwd+loss step shards on the batch axis with no exchange: every rank runs the reference's
B=16 step on its own shard (rank-local SPKD Grams and BN statistics, as a single-GPU Lightning run
would).  The only collective of the training step (config C3) is the student-gradient
all-reduce: ~926 KB fp32, latency-bound over xGMI, so it is issued as ONE flat bucket.
`backend="nccl"` is RCCL on ROCm; the same code runs on gloo for CPU tests.
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend="nccl", device=None):
    rank, world, _ = env_rank()
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, **kw)
    return rank, world


def shard_seed(base_seed, rank):
    """Seed of this rank's synthetic shard: disjoint, reproducible per rank."""
    return int(base_seed) + 1000 * (int(rank) + 1)


def max_over_ranks(value, device=None):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def allreduce_mean_flat(tensors):
    """Average `tensors` (e.g. student grads) across ranks with ONE all-reduce of a flat bucket;
    results are written back in place.  Deterministic for a fixed world size."""
    if not (dist.is_initialized() and dist.get_world_size() > 1) or not tensors:
        return tensors
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat.div_(dist.get_world_size())
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n
    return tensors
