"""One process per GPU: variant/gene sharding and the final gather to rank 0.

Variants (and genes) are independent, so each rank takes a contiguous range and computes
it with no data-path collective; the only exchange is the final gather of the per-shift
outputs to rank 0 (``torch.distributed`` backend "nccl" = RCCL over xGMI on MI355X;
"gloo" on CPU for tests), after which rank 0 writes the reference-layout files.
Launch with ``python -m torch.distributed.run --nproc-per-node N ...``.
"""
from __future__ import annotations

import os

import torch


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def local_device(local: int) -> int:
    """The GPU of local rank ``local``: one rank per GPU.  A local rank beyond the visible devices
    (HIP_VISIBLE_DEVICES narrower than --nproc-per-node) is a launch error and raises, instead of
    silently putting two ranks on one GPU (RCCL also rejects duplicate GPUs in a communicator).
    EXPECTO_SHARE_GPUS=1 opts into sharing (local % visible): the multi-rank rehearsals over gloo
    on a one-GPU box."""
    n = torch.cuda.device_count()
    if 0 <= local < n:
        return local
    if n > 0 and os.environ.get("EXPECTO_SHARE_GPUS") == "1":
        return local % n
    raise RuntimeError(f"local rank {local} has no GPU of its own ({n} visible); launch one rank per GPU "
                       f"(or set EXPECTO_SHARE_GPUS=1 to rehearse several ranks on one GPU)")


def init(backend: str | None = None):
    """Initialise the process group when launched with WORLD_SIZE > 1; returns (rank, world, local).
    Backend: the argument, else $EXPECTO_DIST_BACKEND, else "nccl" (RCCL) on a GPU, "gloo" on CPU."""
    import torch.distributed as dist

    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("EXPECTO_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local_device(local))
        dist.init_process_group(backend=backend)
    return rank, world, local


def _single(world: int) -> bool:
    """True when there is nothing to exchange: one rank and no process group.  A process group of
    one rank (the RCCL smoke test on a one-GPU box) still runs the collectives."""
    import torch.distributed as dist

    return world == 1 and not (dist.is_available() and dist.is_initialized())


def shard_range(n: int, rank: int, world: int):
    """Contiguous [lo, hi) range of n items for `rank` (first n % world ranks get one more)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _padded(t: torch.Tensor, dim: int, n_total: int, world: int):
    x = t.movedim(dim, 0).contiguous()
    max_n = max(shard_range(n_total, r, world)[1] - shard_range(n_total, r, world)[0] for r in range(world))
    if x.shape[0] == max_n:
        return x
    pad = torch.zeros((max_n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    return pad


def _unpad(parts, dim: int, n_total: int, world: int):
    pieces = []
    for r in range(world):
        lo, hi = shard_range(n_total, r, world)
        pieces.append(parts[r][: hi - lo])
    return torch.cat(pieces, 0).movedim(0, dim)


def gather_rows(t: torch.Tensor, dim: int, n_total: int, world: int):
    """Gather the shards of `t` along `dim` (contiguous rank ranges of shard_range) to every rank.

    Returns the full tensor (rank order = global order).  One all_gather of equally padded
    shards (RCCL ring over xGMI on the GPU)."""
    import torch.distributed as dist

    if _single(world):
        return t
    pad = _padded(t, dim, n_total, world)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return _unpad(parts, dim, n_total, world)


def gather_rows_to(t: torch.Tensor, dim: int, n_total: int, world: int, rank: int, dst: int = 0):
    """Gather the shards of `t` along `dim` to rank `dst` only (None on the other ranks).

    The file-writing rank is the only one that needs the full tensor: one RCCL gather moves
    each shard once over xGMI into `dst`, and no other rank allocates the full size."""
    import torch.distributed as dist

    if _single(world):
        return t
    pad = _padded(t, dim, n_total, world)
    if pad.is_cuda and dist.get_backend() == "gloo":
        pad = pad.cpu()       # gloo gathers host tensors only (CPU tests, one-GPU rehearsals)
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, parts, dst=dst)
    return _unpad(parts, dim, n_total, world) if rank == dst else None


def gather_blocks_to(t: torch.Tensor, dim: int, counts, world: int, rank: int, dst: int = 0):
    """Gather variable-size blocks along `dim` to rank `dst`: rank r holds counts[r] rows (a
    streamed batch of its shard; 0 allowed).  Blocks are padded to max(counts) for one gather
    (RCCL on the GPU, gloo on the host); returns the list of rank blocks (rank order) on `dst`,
    None elsewhere."""
    import torch.distributed as dist

    if _single(world):
        return [t]
    m = max(counts)
    x = t.movedim(dim, 0)
    if x.shape[0] != counts[rank]:
        raise ValueError(f"rank {rank} holds {x.shape[0]} rows, counts say {counts[rank]}")
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: x.shape[0]] = x
    if pad.is_cuda and dist.get_backend() == "gloo":
        pad = pad.cpu()       # gloo gathers host tensors only (CPU tests, one-GPU rehearsals)
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, parts, dst=dst)
    if rank != dst:
        return None
    return [parts[r][: counts[r]].movedim(0, dim) for r in range(world)]
