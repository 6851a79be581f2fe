#!/usr/bin/env python3
"""Per-segment error of one mlp_grad case against the fp32 oracle (tests/test_kernels_fuzz_gpu.py
reproduces hypothesis draws with the same generator order).

    python tools/grad_fuzz_probe.py --head 0 --D 1 --A 5 --H 128 --B 45 --seed 1000000
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from relayrl_prototype_amd.ops import GradHead, MLPSpec, mlp_grad  # noqa: E402
from relayrl_prototype_amd.ops import reference as ref  # noqa: E402


def case(head, D, A, H, B, seed, dev):
    g = torch.Generator().manual_seed(seed)
    Aeff = 1 if head == GradHead.VALUE_MSE else A
    sp = MLPSpec(D, H, Aeff)
    pp = sp.init(g)
    X = torch.randn(B, D, generator=g)
    act = torch.randint(0, A, (B,), dtype=torch.int32, generator=g)
    adv = torch.randn(B, generator=g)
    ret = torch.randn(B, generator=g)
    logp_old = -torch.rand(B, generator=g) * 2
    stats = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(B))])
    kw = dict(act=act, adv=adv, ret=ret, logp_old=logp_old, adv_stats=stats, clip_eps=0.2, ent_coef=0.01)
    g_ref, _ = ref.mlp_grad_ref(int(head), pp, X, A, H, None, **kw)
    g64, _ = ref.mlp_grad_ref(int(head), pp, X, A, H, None, dtype=torch.float64,
                              **{k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v)
                                 for k, v in kw.items()})
    slab, _ = mlp_grad(head, pp.to(dev), X.to(dev), A, H, None,
                       **{k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in kw.items()})
    gk = slab.sum(0).double().cpu()
    out = {"head": int(head), "D": D, "A": A, "H": H, "B": B, "seed": seed, "scale": g64.abs().max().item()}
    o = sp.offsets()
    ends = [("w1", o["b1"]), ("b1", o["w2"]), ("w2", o["b2"]), ("b2", o["w3"]), ("w3", o["b3"]), ("b3", sp.P)]
    start = 0
    for name, end in ends:
        seg = slice(start, end)
        out[name] = {"kernel_vs_f64": (gk[seg] - g64[seg].double()).abs().max().item(),
                     "fp32oracle_vs_f64": (g_ref[seg].double() - g64[seg].double()).abs().max().item(),
                     "max_abs": g64[seg].abs().max().item()}
        start = end
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--head", type=int, default=0)
    ap.add_argument("--D", type=int, default=1)
    ap.add_argument("--A", type=int, default=5)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--B", type=int, default=45)
    ap.add_argument("--seed", type=int, default=1000000)
    ap.add_argument("--sweep", action="store_true", help="also nearby seeds / D / B")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    print(json.dumps(case(GradHead(a.head), a.D, a.A, a.H, a.B, a.seed, dev)), flush=True)
    if a.sweep:
        for D in (1, 2, 3):
            for B in (45, 64, 300):
                for s in range(3):
                    r = case(GradHead(a.head), D, a.A, a.H, B, s, dev)
                    worst = max(r[k]["kernel_vs_f64"] / max(r["scale"], 1e-12) for k in ("w1", "b1", "w2", "b2", "w3", "b3"))
                    ref32 = max(r[k]["fp32oracle_vs_f64"] / max(r["scale"], 1e-12)
                                for k in ("w1", "b1", "w2", "b2", "w3", "b3"))
                    print(json.dumps({"D": D, "B": B, "seed": s, "kernel_rel": worst, "fp32_oracle_rel": ref32}),
                          flush=True)


if __name__ == "__main__":
    main()
