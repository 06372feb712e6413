"""GPU: the N-rank path on the one-GPU box (config c4's machinery below RCCL).

* `generate_sharded` in two processes sharing cuda:0 (collectives over gloo on host tensors;
  RCCL refuses two ranks on one device): the free-running greedy copy-head fixture (3 utterances,
  shards of 2 + 1, row_base = global index) gathered on every rank equals the reference's codes
  bit for bit -- the same codes the single-process test checks, so sharding changes nothing.
* `bench.py --gpus 2` under ZK_BENCH_SHARE_GPU=1: the launcher starts two ranks, each runs its
  shard through the library path, the codes are gathered and n_gpus == 2 is reported."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, name, q):
    try:
        import torch
        import torch.distributed as dist

        from tests.golden_util import load_gen_case
        from zonos_amd.distributed import generate_sharded
        from zonos_amd.engine import EngineConfig, HipDecoder
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        c = load_gen_case(name)
        cfg = c["cfg"]
        eng = HipDecoder(EngineConfig(cfg.d_model, cfg.n_layer, cfg.n_heads, cfg.n_kv, cfg.d_ff, cfg.eps), c["W"],
                         "cuda:0")
        local, allc = generate_sharded(eng, c["cond"].cuda(), c["prefix"].cuda(), c["max_new"], 2.0, c["B"], c["sp"],
                                       seed=c["seed"], coll_device="cpu", return_local=True, poll_every=5)
        ok = len(allc) == c["B"] and all(
            np.array_equal(x.cpu().numpy(), c["codes"][i, :, :int(c["lens"][i])]) for i, x in enumerate(allc))
        q.put((rank, ok, len(local), [int(x.shape[1]) for x in allc]))
        dist.destroy_process_group()
    except Exception as e:       # report instead of hanging the parent
        q.put((rank, False, -1, repr(e)))


@pytest.mark.parametrize("name", ["copy_greedy", "copy_eos"])
def test_generate_sharded_two_ranks_bit_identical(name):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, name, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] for r in res), res
    assert [r[2] for r in res] == [2, 1], res          # contiguous shards of 3 utterances


def test_bench_two_ranks_share_gpu():
    env = dict(os.environ, ZK_BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--layers", "2", "--batch", "2", "--lc", "16", "--prefix", "0", "--new-tokens", "24",
                        "--no-dac", "--no-cpu-baseline"], capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4 and d["config"]["parallelism"] == "dp2"
    # 2 ranks x 2 utterances x 24 frames x 9 codebooks in the timed step
    assert abs(d["value"] - 2 * 2 * 24 * 9 / (d["ms_per_step"] / 1e3)) / d["value"] < 0.01
