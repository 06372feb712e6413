"""Batch sharding across GPUs (one process per GPU) and the final codes gather.

SURVEY.md §8(e): utterances are independent, so the batch is split into contiguous blocks
per rank (each rank keeps its own cond+uncond row pairs); the engine's noise stream is keyed
by the global utterance index (row_base), so the codes equal a single-GPU batch. The only
collective is one all_gather of the int32 codes + lengths at the end (RCCL over xGMI on the
GPU box, gloo in the CPU tests)."""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard(global_batch: int, world: int, rank: int) -> tuple[int, int]:
    """(row_base, local_batch) of contiguous utterance blocks; sizes differ by at most 1."""
    base, rem = divmod(global_batch, world)
    local = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, local


def gather_codes(codes: list, device=None, group=None) -> list:
    """All-gather a list of int [9, T_i] code tensors from every rank (rank order = global
    utterance order). Codes travel as int32 (values <= 1025) padded to the max length."""
    world = dist.get_world_size(group)
    device = device or (codes[0].device if codes else torch.device("cpu"))
    n = torch.tensor([len(codes)], device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    lens = torch.tensor([int(c.shape[1]) for c in codes] or [0], device=device)
    tmax = torch.tensor([int(lens.max())], device=device)
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX, group=group)
    nmax = max(int(x) for x in ns)
    T = int(tmax)
    buf = torch.zeros(nmax, 9, max(T, 1), dtype=torch.int32, device=device)
    lb = torch.zeros(nmax, dtype=torch.int64, device=device)
    for i, c in enumerate(codes):
        buf[i, :, : c.shape[1]] = c.to(torch.int32)
        lb[i] = c.shape[1]
    bufs = [torch.empty_like(buf) for _ in range(world)]
    lbs = [torch.empty_like(lb) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    dist.all_gather(lbs, lb, group=group)
    out = []
    for r in range(world):
        for i in range(int(ns[r])):
            out.append(bufs[r][i, :, : int(lbs[r][i])].to(torch.int64))
    return out
