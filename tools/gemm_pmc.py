"""Standalone launches of the c3 decode-step GEMMs and slab reduces (M = 2B = 128 rows) for PMC
collection, one rocprofv3 pass per counter (MI355X_MICROARCH.md, HBM section):

    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/gpmc_f -o run --output-format csv -- python3 tools/gemm_pmc.py
    rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/gpmc_w -o run --output-format csv -- python3 tools/gemm_pmc.py
    python tools/gemm_pmc.py --summary gpurun_out/gpmc_f gpurun_out/gpmc_w --json profiles/r5_gemm_pmc.json

Each GEMM runs 10 times over enough weight copies to exceed the 256 MB Infinity Cache (every launch
streams its weights from HBM, as in the decode step, where 3.2 GB of weights pass between two uses).
The k_resid_ln launches reduce the out_proj (4) / fc2 (8) slabs of a fresh buffer each time.
Algorithmic bytes: weights + activation read once + output (fp32 slabs or bf16 rows)
written once; a reduce: slabs + residual row read, residual + LayerNorm rows written."""
import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

M, D, F, H, HKV, HD, NH = 128, 2048, 8192, 16, 4, 128, 9 * 1026


def specs():
    """(name, kernel-name prefix, N, K, nsplit, mode) of the c3 decode GEMMs (engine split rules)."""
    from zonos_amd.engine import _split_for
    nq = (H + 2 * HKV) * HD
    return [("in_proj", nq, D, _split_for(nq, D, M), 0), ("out_proj", D, H * HD, _split_for(D, H * HD, M, 128), 0),
            ("fc1", 2 * F, D, 1, 1), ("fc2", D, F, _split_for(D, F, M), 0), ("heads", NH, D, 1, 0)]


def alg_bytes(N, K, ns, mode):
    out = M * N * 4 * ns if mode == 0 else M * (N // 2) * 2
    return N * K * 2 + M * K * 2 + out


def reduce_bytes(ns):
    return ns * M * D * 4 + M * D * 2 + 2 * D * 2 + 2 * M * D * 2


def run():
    import torch

    from zonos_amd import _lib
    from zonos_amd._lib import call, ptr
    _lib.load()
    dev = torch.device("cuda")
    S = _lib.stream_ptr()
    for name, N, K, ns, mode in specs():
        ncopy = max(3, int(600e6 // (N * K * 2)) + 1)
        Ws = [torch.randn((N + 63) // 64 * 64, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        part = torch.empty(ns * M * N, device=dev)
        out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
        for i in range(10):
            call("zk_gemm_bf16", ptr(A), K, ptr(Ws[i % ncopy]), M, N, K, ns, mode, ptr(part), ptr(out), None, S)
        torch.cuda.synchronize()
        print(json.dumps(dict(name=name, N=N, K=K, nsplit=ns, mode=mode, alg=alg_bytes(N, K, ns, mode))), flush=True)
        del Ws
    for ns in (4, 8):
        parts = [torch.randn(ns * M * D, device=dev) for _ in range(8)]
        x = torch.randn(M, D, device=dev).to(torch.bfloat16)
        xn = torch.empty_like(x)
        w, b = torch.ones(D, device=dev).to(torch.bfloat16), torch.zeros(D, device=dev).to(torch.bfloat16)
        for i in range(10):
            call("zk_resid_ln", ptr(parts[i % 8]), ns, ptr(x), ptr(w), ptr(b), 1e-5, M, D, ptr(x), ptr(xn), 0, None, S)
        torch.cuda.synchronize()
        print(json.dumps(dict(name=f"resid_ln{ns}", nsplit=ns, alg=reduce_bytes(ns))), flush=True)


def summary(dirs, out_json):
    """Mean FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch of each kernel, matched to the specs by
    the instantiation (each c3 shape has its own k_gemm_ws template arguments)."""
    from collections import defaultdict
    acc = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                acc[(r.get("Kernel_Name", "?"), r["Counter_Name"])].append(float(r["Counter_Value"]))
    # kernel name -> spec by launch order: the specs launch in a fixed order, one instantiation each
    names = []
    for (kn, cn) in acc:
        if ("k_gemm_ws" in kn or "k_resid_ln" in kn) and kn not in names:
            names.append(kn)
    entries = []
    sp = {s[0]: s for s in specs()}
    for kn in names:
        f = acc.get((kn, "FETCH_SIZE"), [0.0])
        w = acc.get((kn, "WRITE_SIZE"), [0.0])
        hbm = (sum(f) / len(f) * 2 + sum(w) / len(w)) * 1024
        short = kn.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        entries.append(dict(kernel=short, fetch_bytes=sum(f) / len(f) * 2 * 1024, write_bytes=sum(w) / len(w) * 1024,
                            hbm_bytes_per_launch=hbm))
    # match by template arguments (k_gemm_ws<MODE, NCH, PF, MT, NCW, ...>: NCH = K / nsplit / 64)
    out = []
    for e in entries:
        k = e["kernel"]
        for name, N, K, ns, mode in sp.values():
            if k.startswith(f"k_gemm_ws<{mode}, {K // ns // 64},"):
                if name == "heads" and ", 3, 1, 2>" not in k:
                    continue
                if name == "in_proj" and ", 4, 1, 2>" not in k:
                    continue
                if name == "out_proj" and ", 2, 1, 2>" not in k:
                    continue
                e.update(name=name, M=M, N=N, K=K, nsplit=ns, alg_bytes=alg_bytes(N, K, ns, mode))
        for ns in (4, 8):
            if k.startswith(f"k_resid_ln_d2k512<{ns},"):
                e.update(name=f"resid_ln{ns}", M=M, N=D, nsplit=ns, alg_bytes=reduce_bytes(ns))
        if "name" in e:
            e["traffic_ratio"] = round(e["hbm_bytes_per_launch"] / e["alg_bytes"], 3)
            out.append(e)
            print(f"{e['name']:10s} {k[:48]:48s} alg {e['alg_bytes'] / 1e6:8.2f} MB  HBM {e['hbm_bytes_per_launch'] / 1e6:8.2f} MB"
                  f"  (fetch {e['fetch_bytes'] / 1e6:7.2f}, write {e['write_bytes'] / 1e6:7.2f})  ratio {e['traffic_ratio']}")
    if out_json:
        json.dump(out, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summary", nargs="*")
    ap.add_argument("--json")
    a = ap.parse_args()
    if a.summary:
        summary(a.summary, a.json)
    else:
        run()
