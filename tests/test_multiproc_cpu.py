"""CPU, world_size 2 (gloo): batch sharding + codes gather used by bench.py on N GPUs."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from zonos_amd.distributed import gather_codes, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 5
    start, local = shard(B, world, rank)
    g = torch.Generator().manual_seed(0)
    full = [torch.randint(0, 1026, (9, 3 + 2 * i), generator=g) for i in range(B)]
    mine = full[start:start + local]
    got = gather_codes(mine)
    q.put((rank, all(torch.equal(a, b) for a, b in zip(got, full)) and len(got) == B))
    dist.destroy_process_group()


def test_shard_partition():
    for B in (1, 7, 64, 512):
        for w in (1, 2, 8):
            parts = [shard(B, w, r) for r in range(w)]
            assert sum(p[1] for p in parts) == B
            assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(w - 1))


def test_gather_codes_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


class StubEngine:
    """Stands in for HipDecoder.generate: utterance b's codes are a function of its global index
    (row_base + b), the seed and ITS cond / uncond rows only, as the real engine's are."""

    def generate(self, cond, prefix, max_new, cfg_scale, B, sp, *, seed, row_base=0, **kw):
        assert cond.shape[0] == 2 * B and (prefix is None or prefix.shape[0] == B)
        out = []
        for b in range(B):
            g = row_base + b
            v = int(cond[b, 0, 0]) * 1000 + int(cond[B + b, 0, 0]) + (seed % 97) + (0 if prefix is None else int(prefix[b, 0, 0]))
            out.append(torch.full((9, 2 + g % 3), v % 1024, dtype=torch.int64))
        return out


def _global_inputs(B):
    cond = torch.zeros(2 * B, 3, 4)
    cond[:B, 0, 0] = torch.arange(B).float()            # cond row i carries i
    cond[B:, 0, 0] = 100 + torch.arange(B).float()      # its uncond partner carries 100 + i
    prefix = torch.arange(B).view(B, 1, 1).expand(B, 9, 2).clone()
    return cond, prefix


def _sharded_worker(rank, world, port, q):
    from zonos_amd.distributed import generate_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(1234 + rank)                      # differs per rank: seed=None must be broadcast
    B = 5
    cond, prefix = _global_inputs(B)
    got = generate_sharded(StubEngine(), cond, prefix, 8, 2.0, B, {}, coll_device="cpu")
    ref = StubEngine().generate(cond, prefix, 8, 2.0, B, {}, seed=0, row_base=0)
    # same codes as one batch up to the seed term, which every rank must share
    seeds = {int(a[0, 0] - b[0, 0]) % 1024 for a, b in zip(got, ref)}
    ok = len(got) == B and len(seeds) == 1 and all(a.shape == b.shape for a, b in zip(got, ref))
    # explicit seed, rank-local inputs, no gather
    rb, n = shard(B, world, rank)
    loc = torch.cat([cond[rb:rb + n], cond[B + rb:B + rb + n]])
    mine = generate_sharded(StubEngine(), loc, prefix[rb:rb + n], 8, 2.0, B, {}, seed=7, gather=False,
                            local_input=True, coll_device="cpu")
    ref7 = StubEngine().generate(cond, prefix, 8, 2.0, B, {}, seed=7)[rb:rb + n]
    ok = ok and len(mine) == n and all(torch.equal(a, b) for a, b in zip(mine, ref7))
    q.put((rank, ok))
    dist.destroy_process_group()


def test_generate_sharded_gloo_world2():
    """generate_sharded over 2 gloo ranks (B = 5: ragged 3 + 2 shards) returns the one-batch codes
    in global order on every rank; seed=None is drawn once and broadcast."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def _default_args_worker(rank, world, port, q):
    """The documented call: no seed, no coll_device, and B < world so rank 1's shard is empty."""
    from zonos_amd.distributed import collective_device, generate_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(99 + rank)
    B = 1
    cond, prefix = _global_inputs(B)
    got = generate_sharded(StubEngine(), cond, prefix, 8, 2.0, B)
    ref = StubEngine().generate(cond, prefix, 8, 2.0, B, {}, seed=0, row_base=0)
    ok = len(got) == 1 and got[0].shape == ref[0].shape and collective_device() == torch.device("cpu")
    q.put((rank, ok, [tuple(c.shape) for c in got], int(got[0][0, 0]) if got else None))
    dist.destroy_process_group()


def test_generate_sharded_default_args_empty_shard():
    """seed=None, coll_device=None, B=1 over 2 ranks (one empty shard) -- the collectives
    pick the group's device on every rank and both ranks return the same codes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_default_args_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] for r in res), res
    assert res[0][3] == res[1][3], res


def test_generate_sharded_single_process():
    from zonos_amd.distributed import generate_sharded
    cond, prefix = _global_inputs(4)
    got = generate_sharded(StubEngine(), cond, prefix, 8, 2.0, 4, {}, seed=3)
    ref = StubEngine().generate(cond, prefix, 8, 2.0, 4, {}, seed=3)
    assert all(torch.equal(a, b) for a, b in zip(got, ref))


class RecordingStub(StubEngine):
    """StubEngine that records the batch each generate() call ran (the GEMM regime is a function of it)."""

    def __init__(self):
        self.batches = []
        self.pads = []

    def generate(self, cond, prefix, max_new, cfg_scale, B, sp, *, seed, row_base=0, **kw):
        self.batches.append(B)
        self.pads.append(kw.pop("pad_rows", 0))
        return super().generate(cond, prefix, max_new, cfg_scale, B, sp, seed=seed, row_base=row_base, **kw)


def _ragged_worker(rank, world, port, q):
    from zonos_amd.distributed import gemm_regime, generate_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 17
    cond, prefix = _global_inputs(B)
    eng = RecordingStub()
    got = generate_sharded(eng, cond, prefix, 8, 2.0, B, {}, seed=5, coll_device="cpu")
    ref = StubEngine().generate(cond, prefix, 8, 2.0, B, {}, seed=5)
    ok = len(got) == B and all(torch.equal(a, b) for a, b in zip(got, ref))
    q.put((rank, ok, eng.batches, [gemm_regime(b) for b in eng.batches], eng.pads))
    dist.destroy_process_group()


def test_generate_sharded_ragged_keeps_one_regime():
    """B = 17 over 2 ranks is a 9 + 8 split, i.e. M = 18 (k_gemm_ws) beside M = 16
    (k_gemv): two reduction orders. The 8-utterance shard is padded to 9, so both ranks run the
    k_gemm_ws regime at the same shape, and the gathered codes are still the one-batch codes. The
    padding utterance is announced to the engine (pad_rows = 1) so it stays out of the EOS protocol
    (the GPU side: tests/test_gpu_generate.py::test_pad_rows_keep_out_of_eos_protocol)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ragged_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] for r in res), res
    assert [r[2] for r in res] == [[9], [9]], res
    assert {g for r in res for g in r[3]} == {"ws"}, res
    assert [r[4] for r in res] == [[0], [1]], res


def test_padded_shard_rule():
    from zonos_amd.distributed import gemm_regime, padded_shard
    for B in (1, 5, 17, 64, 511, 512):
        for w in (1, 2, 3, 8):
            runs = {padded_shard(B, w, r)[2] for r in range(w)} - {0}
            assert len(runs) == 1
            assert all(padded_shard(B, w, r)[2] - padded_shard(B, w, r)[1] <= 1 for r in range(w))
    assert gemm_regime(8) == "gemv" and gemm_regime(9) == "ws" and gemm_regime(64) == "ws" and gemm_regime(65) == "gemm"
