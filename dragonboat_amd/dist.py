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


class RcclComm:
    """An RCCL communicator over the process group's ranks for the C ABI's
    exchange (drb_exchange_rccl*, include/drb_engine.h): what a Go NodeHost
    per GPU would hold (cgo).  Rank 0's ncclUniqueId travels
    over the torch.distributed group; ncclCommInitRank is collective.
    abort() (ncclCommAbort) may be called from another thread to end
    operations that hang."""

    def __init__(self, world, rank):
        import ctypes as C
        import torch.distributed as dist

        class UniqueId(C.Structure):
            _fields_ = [("internal", C.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES
        lib = None
        for name in ("librccl.so.1", "/opt/rocm/lib/librccl.so.1"):
            try:
                lib = C.CDLL(name)
                break
            except OSError:
                pass
        if lib is None:
            raise RuntimeError("librccl not loadable")
        lib.ncclGetUniqueId.argtypes = [C.POINTER(UniqueId)]
        lib.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int,
                                         UniqueId, C.c_int]
        lib.ncclCommDestroy.argtypes = [C.c_void_p]
        lib.ncclCommAbort.argtypes = [C.c_void_p]
        uid = UniqueId()
        if rank == 0 and lib.ncclGetUniqueId(C.byref(uid)) != 0:
            raise RuntimeError("ncclGetUniqueId failed")
        box = [C.string_at(C.addressof(uid), 128) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        C.memmove(C.addressof(uid), box[0], 128)
        self.lib, self.comm = lib, C.c_void_p()
        rc = lib.ncclCommInitRank(C.byref(self.comm), world, uid, rank)
        if rc != 0:
            raise RuntimeError("ncclCommInitRank failed: %d" % rc)

    @property
    def handle(self):
        return self.comm.value

    def abort(self):
        if self.comm.value:
            self.lib.ncclCommAbort(self.comm)
            self.comm.value = None

    def close(self):
        if self.comm.value:
            self.lib.ncclCommDestroy(self.comm)
            self.comm.value = None
