"""Multi-GPU plumbing for the co-resident configurations.

Groups are independent Raft instances, so a node shards them: rank r hosts
groups [r*G, (r+1)*G) -- ShardIDs first_shard_id + g -- with all replicas of
a group on the same GPU, mirroring dragonboat's shardID-partitioned step
workers (internal/server/partition.go:38, engine.go:1270-1299).  There is
no data-path collective: ranks only agree on the tick cadence before timing
and reduce their counters after it.

One process per GPU; the launcher (torch.distributed.run) sets RANK,
WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT.  Backend "nccl" is RCCL on ROCm;
the tests drive the same functions over "gloo" on the CPU.
"""
import os

BASE_SEED = 0x5EEDD8B0


def env():
    return (int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_plan(rank, groups_per_rank, first_shard_id=1):
    """(first_shard_id, seed) of the groups hosted by `rank`."""
    return first_shard_id + rank * groups_per_rank, BASE_SEED ^ rank


def _reduce(value, op, dtype, device):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or \
            dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=dtype, device=device)
    dist.all_reduce(t, op=op)
    return t.item()


def agree_min(value, device="cpu"):
    import torch
    import torch.distributed as dist
    return int(_reduce(int(value), dist.ReduceOp.MIN, torch.int64, device))


def reduce_max(value, device="cpu"):
    import torch
    import torch.distributed as dist
    return float(_reduce(float(value), dist.ReduceOp.MAX, torch.float64,
                         device))


def reduce_sum(value, device="cpu"):
    import torch
    import torch.distributed as dist
    return int(_reduce(int(value), dist.ReduceOp.SUM, torch.int64, device))


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
