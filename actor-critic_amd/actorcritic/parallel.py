"""One process per GPU, data-parallel over env shards.

Each rank steps its own shard of environments (global env ids rank*N_local ..), runs
the rollout and the local forward/backward/K-FAC statistics, and the ranks exchange one
flat buffer per update — [grads | loss scalars | A stats | G stats] — with a single
all-reduce (``torch.distributed`` backend ``nccl`` = RCCL over xGMI on ROCm, ``gloo`` on
CPU for tests).  Parameters, velocities, factors and inverses stay replicated and
bit-identical because every rank applies the same deterministic kernels to the same
reduced buffer.
"""

import os

import torch
import torch.distributed as dist


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def world_size():
    return dist.get_world_size() if is_initialized() else 1


def rank():
    return dist.get_rank() if is_initialized() else 0


def backend_name():
    """'nccl' (= RCCL on ROCm), 'gloo', or None on one process."""
    return dist.get_backend() if is_initialized() else None


def local_rank():
    return int(os.environ.get('LOCAL_RANK', '0'))


def init_from_env(backend=None):
    """Initialises the process group from torchrun's environment (RANK, WORLD_SIZE,
    MASTER_ADDR/PORT, LOCAL_RANK) when WORLD_SIZE > 1; pins the local GPU."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank() % max(1, torch.cuda.device_count()))
    if ws > 1 and not is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if backend is None:
            # ACMI_DIST_BACKEND=gloo rehearses N ranks on one GPU (RCCL refuses
            # two ranks on one device); the default on GPUs is nccl (= RCCL)
            backend = os.environ.get('ACMI_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
        dist.init_process_group(backend=backend, init_method='env://')
    return world_size(), rank()


def allreduce_sum_(t, force=False):
    """In-place SUM over ranks; force: also with a process group of one rank (the
    engine's ACMI_FORCE_COLLECTIVE test switch)."""
    if world_size() > 1 or (force and is_initialized()):
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def allreduce_sum_async(t):
    """Starts an in-place SUM all-reduce; the returned work's wait() makes the current
    stream wait for it (RCCL/NCCL runs collectives on its own stream)."""
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)


def broadcast_(t, src=0):
    if world_size() > 1:
        dist.broadcast(t, src)
    return t


def barrier():
    if world_size() > 1:
        if dist.get_backend() == 'nccl':
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def max_over_ranks(x, device=None):
    if world_size() == 1:
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, device=None):
    if world_size() == 1:
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def destroy():
    if is_initialized():
        dist.destroy_process_group()
