"""The reference's own sampling noise on the GPU: torch's `Tensor.exponential_(1)` stream
(zonos/sampling.py:26-28), reproduced by the HIP sampler (noise mode "torch", zk_torch_exponential /
zk_sample_logits_torch / zk_gen_state.noise_*) and checked against torch itself on this device."""
import numpy as np
import pytest
import torch

from oracle import torch_philox, zonos_ref

from .golden_util import load_gen_case
from .test_gpu_generate import TAU_LOGIT, TAU_LOGRATIO, _engine, _margins

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from zonos_amd import _lib
    _lib.load()


# sizes: tiny, one [B][9][1026] tensor at B = 1 / 3 / 64 (the c3 sampler call: grid-capped) / 300
# (two iterations of torch's grid-stride loop)
SIZES = (17, 9 * 1026, 3 * 9 * 1026, 64 * 9 * 1026, 300 * 9 * 1026)


@pytest.mark.parametrize("seed", [0, 421, 2 ** 40 + 7])
def test_noise_bit_identical_to_torch(seed):
    """zk_torch_exponential == torch's own exponential_ for the same generator state, bit for bit,
    over consecutive calls (the offset advancing as torch advances it)."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.sampling import torch_noise_policy
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    for n in SIZES + SIZES[::-1]:
        off = int(g.get_offset())
        ref = torch.empty(n, device=DEV).exponential_(1, generator=g)
        stride, incr = torch_noise_policy(n, DEV)
        assert int(g.get_offset()) == off + incr, (n, off, g.get_offset(), incr)
        out = torch.empty(n, device=DEV)
        call("zk_torch_exponential", ptr(out), n, seed, off, stride, stream_ptr(torch.device(DEV)))
        torch.cuda.synchronize()
        bad = int((out.view(torch.int32) != ref.view(torch.int32)).sum())
        assert bad == 0, f"n={n} offset={off}: {bad} values differ"


def test_policy_matches_oracle_and_device():
    from zonos_amd.sampling import torch_noise_policy
    p = torch.cuda.get_device_properties(0)
    for n in SIZES + (1, 256, 257, 2 ** 21, 2 ** 21 + 1):
        assert torch_noise_policy(n, DEV) == torch_philox.policy(n, p.multi_processor_count,
                                                                 p.max_threads_per_multi_processor)


@pytest.mark.parametrize("B", [4, 64, 300])
def test_sample_from_logits_default_is_the_reference_stream(B):
    """sample_from_logits without a seed races against exactly the noise torch's exponential_
    would give the reference on this generator state, and leaves the generator where that call
    leaves it; greedy calls draw nothing. Tokens = the oracle sampler (the reference's
    algorithm, pinned by sampler.npz) fed that noise; fp32 softmax/exp differ in the last ulp
    between CPU and GPU, so at most 1 flipped token per 2,000 (test_sampler_golden_exact allows 1 in its
    cases). B = 64: the c3 sampler call (torch's grid capped at 2048 blocks); B = 300: two iterations of
    torch's grid-stride loop (an 8-offset call)."""
    from zonos_amd.sampling import sample_from_logits
    K, V = 9, 1026
    gen = torch.Generator().manual_seed(5)
    logits = (torch.randn(B, K, V, generator=gen) * 3).to(DEV)
    hist = torch.randint(0, 1024, (B, K, 12), generator=gen).to(DEV)
    cases = [dict(temperature=1.0, linear=0.65, conf=0.4, quad=0.0), dict(temperature=0.8, top_p=0.9, top_k=50,
             min_p=0.05), dict(temperature=1.0)]
    flips = 0
    g = torch.cuda.default_generators[0]
    for i, sp in enumerate(cases):
        torch.manual_seed(100 + i)
        off0 = int(g.get_offset())
        tok = sample_from_logits(logits, generated_tokens=hist, repetition_penalty=2.5, repetition_penalty_window=8,
                                 **sp).squeeze(-1).cpu()
        off1 = int(g.get_offset())
        torch.manual_seed(100 + i)
        q = torch.empty(B, K, V, device=DEV).exponential_(1)
        assert off1 == int(g.get_offset()) and off1 > off0, (off0, off1, int(g.get_offset()))
        exp = zonos_ref.sample(logits.cpu(), q.cpu(), generated_tokens=hist.cpu(), repetition_penalty=2.5,
                               repetition_penalty_window=8, **sp).squeeze(-1)
        flips += int((tok != exp).sum())
    assert flips <= max(1, 3 * B * K // 2000), flips
    torch.manual_seed(7)
    off0 = int(g.get_offset())
    sample_from_logits(logits, temperature=0.0)
    assert int(g.get_offset()) == off0


def _eos_near_tie(tr, tau) -> bool:
    """Some codebook-0 draw of the oracle's run, on a row that has not stopped yet (model.py:399-402:
    later EOS decisions of a stopped row change nothing), has EOS among its top two with a margin
    <= tau."""
    stopped = torch.zeros(tr["tokens"][0].shape[0], dtype=torch.bool)
    for dec, tok in zip(tr["decision"], tr["tokens"]):
        for kind, arr in dec:
            top = arr[:, 0].topk(2, dim=-1)
            m = torch.log(top.values[:, 0] / top.values[:, 1].clamp_min(1e-38))
            eos = (top.indices == 1024).any(dim=-1)
            if bool((eos & (m <= tau) & ~stopped).any()):
                return True
        stopped |= tok[:, 0, 0] == 1024
    return False


MAX_REJECTED = {"sampled_cli": 3, "eos_sampled": 12, "sampled_knobs": 3}


@pytest.mark.parametrize("name", ["sampled_cli", "eos_sampled", "sampled_knobs"])
def test_generate_reference_noise_teacher_forced(name):
    """generate() with the reference's noise (Zonos.generate's default): the oracle's generate (the
    reference's loop, pinned by the golden fixtures) run on the CPU with its sampler noise drawn from
    torch's CUDA generator call by call -- exactly the reference's draws -- and the engine fed that
    history (teacher forcing) take the same decision at every (step, utterance, codebook) whose margin
    clears the tolerance of test_generate_teacher_forced_matches_reference, and leave the generator at
    the same offset (the same number of sampler calls, EOS resamples included)."""
    c = load_gen_case(name)
    B = c["B"]
    sp = c["sp"]
    gain = (sp["linear"] + np.log(1026) * sp["conf"]) if sp["linear"] > 0 else 1.0
    tau_ratio = TAU_LOGRATIO * max(1.0, gain) / max(sp["temperature"], 1e-6)
    # A codebook-0 decision between EOS and another token whose margin is within the tolerance may
    # go either way on the GPU; it changes that row's EOS state and the number of sampler calls
    # (a resample), i.e. the noise of every later step. Use the first generator seed whose
    # reference run has no such decision, so every step stays comparable. The rejected seeds are
    # counted and bounded per fixture. The count is deterministic (torch's generator,
    # the CPU oracle); MAX_REJECTED holds the measured count plus a margin of two, so a looser
    # tolerance or a changed fixture that excludes more runs fails here. eos_sampled is the EOS
    # fixture: every row ends on a sampled EOS and EOS sits in codebook 0's top two on many steps
    # of every row, so most seeds carry a near-tie somewhere (10 rejected before seed 4331,
    # profiles/r6_final_gpu_tests.log); the two other fixtures pass within a few seeds.
    rejected = 0
    for seed in range(4321, 4521):
        g = torch.Generator(device=DEV)
        g.manual_seed(seed)
        calls = []

        def noise_fn(step, draw):
            calls.append((step, draw))
            return torch.empty(B, 9, 1026, device=DEV).exponential_(1, generator=g).cpu()

        tr = {}
        zonos_ref.generate(c["W"], c["cfg"], c["cond"], c["prefix"], c["max_new"], 2.0, B, sp, trace=tr,
                           noise_fn=noise_fn)
        if not _eos_near_tie(tr, tau_ratio):
            break
        rejected += 1
    else:
        pytest.fail("no generator seed without an EOS near-tie")
    print(f"{name}: generator seed {seed}, {rejected} seed(s) rejected for an EOS near-tie")
    assert rejected <= MAX_REJECTED[name], (name, rejected)
    off_ref = int(g.get_offset())
    gold = tr["delayed"].long()
    P = c["prefix"].shape[2]
    stats = dict(checked=0, skipped=0, mismatch=[])

    def check(frame, step):
        if frame.shape[2] == 0:
            return
        off = P + 1 + step
        got, exp = frame.cpu(), gold[..., off:off + 1]
        m = _margins(tr["decision"][step])
        tau = TAU_LOGIT if tr["decision"][step][-1][0] == "logit" else tau_ratio
        for b in range(B):
            for k in range(9):
                if m[b, k] <= tau:
                    stats["skipped"] += 1
                    continue
                stats["checked"] += 1
                if int(got[b, k, 0]) != int(exp[b, k, 0]):
                    stats["mismatch"].append((step, b, k, int(got[b, k, 0]), int(exp[b, k, 0]), float(m[b, k])))
        frame.copy_(exp.to(frame.device))

    g2 = torch.Generator(device=DEV)
    g2.manual_seed(seed)
    eng = _engine(c["W"], c["cfg"])
    eng.generate(c["cond"].cuda(), c["prefix"].cuda(), c["max_new"], 2.0, B, sp, noise="torch", generator=g2,
                 callback=lambda f, s, n: (check(f, s), True)[1], _after_prefill=lambda f: check(f, 0))
    thresholds = sp.get("top_p", 0) > 0 or sp.get("min_p", 0) > 0
    allowed = stats["checked"] // 200 if thresholds else 0
    assert len(stats["mismatch"]) <= allowed, stats["mismatch"][:10]
    frac = stats["skipped"] / (stats["checked"] + stats["skipped"])
    print(name, "seed", seed, len(calls), "sampler calls;", {k: (v if k != "mismatch" else len(v)) for k, v in stats.items()})
    assert frac <= 0.5, frac
    assert int(g2.get_offset()) == off_ref, (int(g2.get_offset()), off_ref, len(calls))


def test_generate_reference_noise_graph_equals_eager():
    """The hipGraph replay and the eager launches of the torch-noise step give the same codes and
    leave the generator at the same offset."""
    c = load_gen_case("eos_sampled")
    eng = _engine(c["W"])
    outs, offs = [], []
    for graph, poll in ((True, 7), (False, 1)):
        g = torch.Generator(device=DEV)
        g.manual_seed(99)
        outs.append(eng.generate(c["cond"].cuda(), c["prefix"].cuda(), c["max_new"], 2.0, c["B"], c["sp"],
                                 noise="torch", generator=g, use_graph=graph, poll_every=poll))
        offs.append(int(g.get_offset()))
    assert offs[0] == offs[1]
    assert all(torch.equal(x, y) for x, y in zip(*outs))


def test_hybrid_reference_noise_graph_equals_eager():
    """The hybrid engine (HybridDecoder shares generate()) with the reference's noise: graph replay ==
    eager launches, codes and generator offset; the offset advanced by (prefill + steps + resamples)
    calls of the [B][9][1026] policy increment."""
    from oracle import hybrid_ref as HR

    from .test_gpu_hybrid import TINYH
    from .test_gpu_hybrid import _engine as hybrid_engine
    from zonos_amd.sampling import torch_noise_policy
    W = HR.make_weights(TINYH, seed=2, head_scale=4.0)
    B, Lc, P, new = 3, 12, 4, 20
    cond = zonos_ref.synthetic_conditioning(B, Lc, TINYH.d_model).to(DEV)
    prefix = zonos_ref.synthetic_prefix_codes(B, P).to(DEV)
    sp = dict(temperature=1.0, top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
              repetition_penalty_window=8)
    eng = hybrid_engine(W)
    _, incr = torch_noise_policy(B * 9 * 1026, DEV)
    outs, offs = [], []
    for graph, poll in ((True, 6), (False, 1)):
        g = torch.Generator(device=DEV)
        g.manual_seed(77)
        outs.append(eng.generate(cond, prefix, new, 2.0, B, sp, noise="torch", generator=g, use_graph=graph,
                                 poll_every=poll))
        offs.append(int(g.get_offset()))
    assert offs[0] == offs[1] and offs[0] % incr == 0 and offs[0] // incr >= new, (offs, incr)
    assert all(torch.equal(x, y) for x, y in zip(*outs))
