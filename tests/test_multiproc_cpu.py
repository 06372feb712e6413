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
