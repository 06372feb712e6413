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


def collective_device(group=None) -> torch.device:
    """The device a collective of ``group`` runs on: the current GPU for an nccl (RCCL) group,
    which has no CPU backend, else the CPU (gloo). Every rank must pass tensors on the same kind of
    device, whatever its shard holds, so this depends on the group only."""
    backend = str(dist.get_backend(group)).lower()
    if "nccl" in backend:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_codes(codes: list, device=None, group=None) -> list:
    """All-gather a list of int [9, T_i] code tensors from every rank (rank order = global
    utterance order). Codes travel as int32 (values <= 1025) padded to the max length.
    ``device`` None picks the group's collective device (`collective_device`), also on a rank
    whose shard is empty."""
    world = dist.get_world_size(group)
    device = torch.device(device) if device is not None else collective_device(group)
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


def gemm_regime(batch: int) -> str:
    """The decode GEMM regime of a batch of utterances (2 CFG rows each), DESIGN.md §4: split counts
    depend on (N, K) only, but the reduction ORDER differs between regimes -- ``"gemv"`` (M <= 16,
    k_gemv_* K quarters), ``"ws"`` (16 < M <= 128, k_gemm_ws sequential K), ``"gemm"`` (M > 128)."""
    m = 2 * batch
    return "gemv" if m <= 16 else ("ws" if m <= 128 else "gemm")


def padded_shard(global_batch: int, world: int, rank: int) -> tuple[int, int, int]:
    """(row_base, local_batch, run_batch): the rank's contiguous block and the batch it actually
    runs. Blocks differ by at most one utterance, so a ragged split (B = 17 over 2 ranks: 9 + 8)
    would run M = 18 (k_gemm_ws) on one rank and M = 16 (k_gemv) on the other -- two reduction orders.
    Every non-empty block is padded to the largest block size instead, so all ranks run the same
    kernels on the same shapes; an empty block stays empty."""
    row_base, local = shard(global_batch, world, rank)
    most = -(-global_batch // world)
    return row_base, local, (most if local > 0 else 0)


def _pad_rows(x: torch.Tensor, local: int, run: int, cfg_pairs: bool) -> torch.Tensor:
    """Append run - local copies of the last utterance (of each CFG half when ``cfg_pairs``)."""
    if run == local:
        return x
    if not cfg_pairs:
        return torch.cat([x, x[local - 1:local].expand(run - local, *x.shape[1:])])
    c, u = x[:local], x[local:]
    return torch.cat([c, c[-1:].expand(run - local, *x.shape[1:]), u, u[-1:].expand(run - local, *x.shape[1:])])


def _split_rows(cond: torch.Tensor, global_batch: int, row_base: int, local: int) -> torch.Tensor:
    """This rank's CFG rows of a global [2B, Lc, D] conditioning: cond rows [rb, rb+n) and their
    uncond partners [B+rb, B+rb+n) (model.py:113, 213-218 keep each pair B rows apart)."""
    return torch.cat([cond[row_base:row_base + local], cond[global_batch + row_base:global_batch + row_base + local]])


def generate_sharded(model, prefix_conditioning: torch.Tensor, audio_prefix_codes: torch.Tensor | None = None,
                     max_new_tokens: int = 86 * 30, cfg_scale: float = 2.0, batch_size: int = 1,
                     sampling_params: dict | None = None, *, seed: int | None = None, group=None,
                     gather: bool = True, local_input: bool = False, coll_device=None, return_local: bool = False,
                     uniform_shards: bool = True, **generate_kw):
    """Zonos.generate (model.py:224-457) of a GLOBAL batch of ``batch_size`` utterances sharded over
    the ranks of ``group`` (one process per GPU) -- the library form of zonos_batch_cli.py:113-162's
    batching with the batch split across the node's GPUs.

    * Each rank takes a contiguous block of utterances (`shard`); ``row_base`` = the block's global
      index keys the sampling noise, so each utterance's codes do not depend on the rank count
      (within one GEMM regime).
    * ``prefix_conditioning`` is the global [2B, Lc, D] tensor (and ``audio_prefix_codes`` the
      global [B, 9, P]); with ``local_input=True`` they already hold only this rank's rows
      ([2b, Lc, D] / [b, 9, P], b = the rank's share).
    * ``seed`` None draws one seed on rank 0 from torch's generator and broadcasts it.
    * ``coll_device`` None runs the collectives on the group's device (`collective_device`: the
      current GPU under nccl, the CPU under gloo).
    * ``uniform_shards`` (default) pads a block that is one utterance short of the largest block with
      a copy of its last utterance (its codes are dropped), so every rank runs the same GEMM regime
      and shapes (`padded_shard`); an exactly divisible batch (the benchmark's 64 per GPU) pads nothing.
    * No collective touches the decode; with ``gather`` one all_gather of the int32 codes returns
      the global list (utterance order) on every rank, else the rank's own list;
      ``return_local`` returns (the rank's own list on its device, the gathered list).
    ``model`` is a ``zonos_amd.model.Zonos`` or an engine (``HipDecoder`` / ``HybridDecoder``);
    extra keywords go to its ``generate``. Without an initialised process group this is
    ``model.generate`` on the whole batch."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    row_base, local, run = padded_shard(batch_size, world, rank)
    if not uniform_shards or world == 1:
        run = local
    if world > 1 and coll_device is None:
        coll_device = collective_device(group)
    if world > 1 and seed is None:
        s = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64) if rank == 0 else torch.zeros(1, dtype=torch.int64)
        s = s.to(coll_device)
        dist.broadcast(s, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        seed = int(s.item())
    elif seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    cond, prefix = prefix_conditioning, audio_prefix_codes
    if not local_input and world > 1:
        if cond.shape[0] != 2 * batch_size:
            raise ValueError(f"Batch size mismatch: {batch_size} * 2 != {cond.shape[0]}")
        cond = _split_rows(cond, batch_size, row_base, local)
        if prefix is not None:
            prefix = prefix[row_base:row_base + local]
    if local == 0:
        codes = []
    else:
        if run != local:
            cond = _pad_rows(cond, local, run, cfg_pairs=True)
            if prefix is not None:
                prefix = _pad_rows(prefix, local, run, cfg_pairs=False)
        if run != local:                 # the padding rows stay out of the EOS protocol (engine.generate)
            generate_kw = dict(generate_kw, pad_rows=run - local)
        codes = model.generate(cond, prefix, max_new_tokens, cfg_scale, run, sampling_params, seed=seed,
                               row_base=row_base, **generate_kw)[:local]
    if world == 1 or not gather:
        allc = codes
    else:
        allc = gather_codes(codes, device=coll_device, group=group)
    return (codes, allc) if return_local else allc
