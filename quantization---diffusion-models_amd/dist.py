"""Data-parallel denoising across the GPUs of one node.

Prompts are independent, so the batch shards with no per-step collective: one process per GPU
holds a UNet replica (W8A8 SD1.5 ~1.7 GB fp16 buffers; HBM is 288 GB), rank 0 broadcasts the
text embeddings [2B, 77, D] once per generate over RCCL (xGMI), every rank runs its own
50-step graph, and the final latents are gathered to rank 0.  ``torch.distributed`` with the
"nccl" backend is RCCL on ROCm; CPU tests use "gloo" with the same code.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


def shard_range(total, rank, world):
    """Contiguous shard of `total` items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _host_staged():
    """gloo (CPU tests, several ranks sharing one GPU) moves HIP tensors through host memory."""
    return dist.get_backend() != "nccl"


def broadcast_context(ctx, src=0):
    """Broadcast the text-embedding batch from `src` (in place).  No-op at world size 1."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        if ctx.is_cuda and _host_staged():
            h = ctx.cpu()
            dist.broadcast(h, src)
            ctx.copy_(h)
        else:
            dist.broadcast(ctx, src)
    return ctx


def gather_latents(lat, dst=0):
    """Gather equally-shaped per-rank latents to `dst` -> [world * B, ...] (None elsewhere)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return lat
    world = dist.get_world_size()
    if dist.get_backend() == "nccl":
        # a true gather (ProcessGroupNCCL::gather: each rank sends its shard to dst only), not an
        # all_gather that would ship every shard to every rank
        out = [torch.empty_like(lat) for _ in range(world)] if dist.get_rank() == dst else None
        dist.gather(lat.contiguous(), out, dst)
        return torch.cat(out) if dist.get_rank() == dst else None
    src = lat.cpu() if lat.is_cuda else lat
    out = [torch.empty_like(src) for _ in range(world)] if dist.get_rank() == dst else None
    dist.gather(src, out, dst)
    if dist.get_rank() != dst:
        return None
    return torch.cat(out).to(lat.device)


def share_gemm_table(warm_eager, rank=None, world=None):
    """Rank 0 tunes every GEMM shape of the step (`warm_eager()`: one eager step, no collectives)
    and broadcasts its kernel table; the other ranks install it before their own warm-up, so all
    ranks run the same kernel variants and compute bit-identical results for identical inputs
    (the tuner times candidates, and split-K / halo candidates change the fp32 summation order).
    Returns the shared table."""
    from . import kernels as K
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    if world <= 1:
        warm_eager()
        return K.export_table()
    if rank == 0:
        warm_eager()
    box = [K.export_table() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    if rank != 0:
        K.import_table(box[0])
    return box[0]


def shard_context(full_ctx, rank, world):
    """Rows of a [2B, S, D] CFG context (uncond first) for this rank's prompt shard."""
    b = full_ctx.shape[0] // 2
    s, e = shard_range(b, rank, world)
    return torch.cat([full_ctx[s:e], full_ctx[b + s:b + e]])
