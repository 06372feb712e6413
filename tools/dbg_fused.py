import sys, torch
sys.path.insert(0, '.')
from zonos_amd._lib import call, ptr, stream_ptr, load
from zonos_amd.engine import rope_table
load()
DEV = 'cuda'
R, ctx, H, Hk, nsplit, gs = 128, 300, 16, 4, 1, 4
hd = 128; smax = 512
g = torch.Generator(device="cpu").manual_seed(R * 1000 + ctx)
N = (H + 2 * Hk) * hd
part = (torch.randn(gs, R, N, generator=g) * 0.5).to(DEV)
kc0 = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
vt0 = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
freqs = rope_table(16384, hd).to(DEV)
s = stream_ptr()
work = torch.empty(R * Hk * nsplit * (8 + 4 * hd), device=DEV)
kc1, vt1 = kc0.clone(), vt0.clone()
q = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
out1 = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
call("zk_qkv_rope", ptr(part), gs, R, 1, H, Hk, hd, ptr(freqs), ctx - 1, None, ptr(q), ptr(kc1), ptr(vt1), smax, None, None, s)
call("zk_attn_decode", ptr(q), ptr(kc1), ptr(vt1), R, H, Hk, hd, smax, ctx, None, ptr(work), nsplit, ptr(out1), None, s)
def fused(kc, vt):
    o = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
    call("zk_attn_decode_qkv", ptr(part), gs, ptr(freqs), ptr(kc), ptr(vt), R, H, Hk, hd, smax, ctx, None, ptr(work), nsplit, ptr(o), None, s)
    torch.cuda.synchronize()
    return o
a = fused(kc0.clone(), vt0.clone())
b = fused(kc0.clone(), vt0.clone())
c = fused(kc1.clone(), vt1.clone())   # cache already holds the new k/v
out2 = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
call("zk_attn_decode", ptr(q), ptr(kc1), ptr(vt1), R, H, Hk, hd, smax, ctx, None, ptr(work), nsplit, ptr(out2), None, s)
torch.cuda.synchronize()
print("unfused deterministic", torch.equal(out1, out2))
print("fused deterministic", torch.equal(a, b))
print("fused==unfused", torch.equal(a, out1), "fused(prefilled)==unfused", torch.equal(c, out1))
d = (a.float() - out1.float()).abs().view(R, H, hd)
bad = (d > 0).nonzero()
print("n diff", bad.shape[0], "rows", bad[:, 0].unique().tolist()[:20], "heads", bad[:, 1].unique().tolist())
import os
if os.environ.get("ZK_LIB_PATH"):
    w2 = torch.zeros(R * H * hd, device=DEV)
    call("zk_attn_decode_qkv", ptr(part), gs, ptr(freqs), ptr(kc0.clone()), ptr(vt0.clone()), R, H, Hk, hd, smax, ctx, None, ptr(w2), 1, ptr(out2), None, s)
    torch.cuda.synchronize()
    qf = w2.view(torch.bfloat16)[:R * H * hd].view(R, H * hd)
    print("q equal", torch.equal(qf, q), (qf.float() - q.float()).abs().max().item())
    dq = (qf.float() - q.float()).abs().view(R, H, hd)
    nz = (dq > 0).nonzero()
    print("q diffs", nz.shape[0], nz[:10].tolist())
