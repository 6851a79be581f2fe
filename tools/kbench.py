#!/usr/bin/env python3
"""Kernel micro-benchmarks (timed with HIP events, interleaved rounds in one process).

  python tools/kbench.py grad --B 2097152 --iters 20      # fused value fwd+bwd kernel
  python tools/kbench.py all                               # every hot kernel

Usable under rocprofv3 (--kernel-trace / --pmc) to attribute counters to one kernel.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from relayrl_prototype_amd.ops import FwdMode, GradHead, MLPSpec, hip, mlp_forward, mlp_grad, adam_step, gae_scan_tm
from relayrl_prototype_amd.ops import reduce_slabs


STAMP_NAMES = ["xstore+bar", "layer1+bar", "layer2 mfma", "head partials", "bar3", "dout+prefetch",
               "dh2+bar", "dh1 mfma", "dW1", "dW2 mfma"]


def run_stamps(fn, ns, tune, label, rows):
    """Per-segment cycles per 64-row slab of the value-grad kernel (diagnostic stamps build)."""
    dev = torch.device("cuda")
    st = torch.zeros(ns * 8 * 16, dtype=torch.int64, device=dev)
    hip().set_value_grad_stamps(st)
    old_t = hip().set_value_grad_tune(8 | tune)
    fn()
    torch.cuda.synchronize()
    hip().set_value_grad_tune(old_t)
    hip().set_value_grad_stamps(torch.empty(0, device=dev))
    slabs_per_wg = rows / 64 / ns
    seg = st.view(ns, 8, 16).double().mean(0) / slabs_per_wg
    res = {STAMP_NAMES[k]: [round(x, 1) for x in seg[:, k].tolist()] for k in range(10)}
    res["total_w0_w4"] = [round(float(seg[0, :10].sum()), 1), round(float(seg[4, :10].sum()), 1)]
    # once per workgroup, not per slab: kernel entry -> loop, last slab -> kernel end
    per_wg = st.view(ns, 8, 16).double().mean(0)
    res["prologue_per_wg"] = [round(x, 1) for x in per_wg[:, 10].tolist()]
    res["epilogue_per_wg"] = [round(x, 1) for x in per_wg[:, 11].tolist()]
    res["slabs_per_wg"] = slabs_per_wg
    print(json.dumps({"stamps_cycles_per_slab_per_wave": res, "tune": tune, "kernel": label}))


def timeit(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["grad", "pgrad", "pgauss", "fwd", "rollout", "adam", "rslab", "scan", "all"])
    ap.add_argument("--B", type=int, default=2097152)
    ap.add_argument("--vd", type=int, default=4, help="input width of the value-grad bench (grad)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--stamps", action="store_true", help="diagnostic per-segment cycle stamps of the value-grad kernel")
    ap.add_argument("--tunes", default="", help="comma list of value_grad scheduling variants to time too")
    ap.add_argument("--stamp-tunes", default="", help="comma list of tunes to run the stamps build with")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, H, D = a.B, a.H, a.vd
    g = torch.Generator().manual_seed(0)
    X = torch.randn(B, D, generator=g).to(dev)
    ret = torch.randn(B, generator=g).to(dev)
    adv = torch.randn(B, generator=g).to(dev)
    act = torch.randint(0, 2, (B,), generator=g, dtype=torch.int32).to(dev)
    pv = MLPSpec(D, H, 1).init(g).to(dev)
    pp = MLPSpec(D, H, 2).init(g).to(dev)
    res = {}
    flop_row = 2 * (D * H + H * H + H) * 3  # fwd + bwd-data + wgrad (nominal)
    if a.which in ("grad", "all"):
        ns = hip().mlp_grad_slabs(B)
        slab = torch.empty(ns, pv.numel(), device=dev)
        ls = torch.empty(ns, 8, device=dev)
        us = timeit(lambda: mlp_grad(GradHead.VALUE_MSE, pv, X, 1, H, ret=ret, grad_slab=slab, loss_slab=ls), a.iters)
        res["value_grad_us"] = us
        res["value_grad_TFLOPs_nominal"] = flop_row * B / us / 1e6
        stamp_tunes = [0] if a.stamps else []
        if a.stamp_tunes:
            stamp_tunes = [int(x) for x in a.stamp_tunes.split(",")]
        for t in stamp_tunes:
            run_stamps(lambda: mlp_grad(GradHead.VALUE_MSE, pv, X, 1, H, ret=ret, grad_slab=slab, loss_slab=ls),
                       ns, t, "value", B)
        if a.tunes:
            for t in [int(x) for x in a.tunes.split(",")]:
                old_t = hip().set_value_grad_tune(t)
                res[f"value_grad_tune{t}_us"] = timeit(
                    lambda: mlp_grad(GradHead.VALUE_MSE, pv, X, 1, H, ret=ret, grad_slab=slab, loss_slab=ls), a.iters)
                hip().set_value_grad_tune(old_t)
        old = hip().set_value_grad_mode(0)  # the fp32-MFMA kernel, for comparison
        us0 = timeit(lambda: mlp_grad(GradHead.VALUE_MSE, pv, X, 1, H, ret=ret, grad_slab=slab, loss_slab=ls), a.iters)
        hip().set_value_grad_mode(old)
        res["value_grad_fp32mfma_us"] = us0
    if a.which in ("pgrad", "all"):
        ns = hip().mlp_grad_slabs(B)
        slab = torch.empty(ns, pp.numel(), device=dev)
        ls = torch.empty(ns, 8, device=dev)
        st = torch.tensor([0.0, float(B), float(B)], device=dev)
        fpg = lambda: mlp_grad(GradHead.PG_CAT, pp, X, 2, H, act=act, adv=adv, adv_stats=st, grad_slab=slab,  # noqa
                               loss_slab=ls)
        us = timeit(fpg, a.iters)
        res["policy_grad_us"] = us
        if a.stamps:
            run_stamps(fpg, ns, 0, "policy_cat2", B)
        old = hip().set_value_grad_mode(0)
        res["policy_grad_fp32mfma_us"] = timeit(lambda: mlp_grad(GradHead.PG_CAT, pp, X, 2, H, act=act, adv=adv,
                                                                 adv_stats=st, grad_slab=slab, loss_slab=ls), a.iters)
        hip().set_value_grad_mode(old)
    if a.which in ("pgauss", "all"):
        # HalfCheetah PPO policy step: D = 17, A = 6 Gaussian head (bf16x6 kernel vs fp32 MFMA)
        Dg, Ag = 17, 6
        Xg = torch.randn(B, Dg, generator=g).to(dev)
        pg = MLPSpec(Dg, H, Ag, True).init(g).to(dev)
        actc = torch.randn(B, Ag, generator=g).to(dev)
        lpo = -torch.rand(B, generator=g).to(dev) * 5
        ns = hip().mlp_grad_slabs(B)
        slab = torch.empty(ns, pg.numel(), device=dev)
        ls = torch.empty(ns, 8, device=dev)
        st = torch.tensor([0.0, float(B), float(B)], device=dev)
        fn = lambda: mlp_grad(GradHead.PPO_GAUSS, pg, Xg, Ag, H, actc=actc, adv=adv, logp_old=lpo, adv_stats=st,  # noqa
                              grad_slab=slab, loss_slab=ls)
        res["ppo_gauss_split_us"] = timeit(fn, a.iters)
        if a.stamps:
            run_stamps(fn, ns, 0, "ppo_gauss", B)
        old = hip().set_value_grad_mode(0)
        res["ppo_gauss_fp32mfma_us"] = timeit(fn, a.iters)
        hip().set_value_grad_mode(old)
        Xv = Xg
        pv17 = MLPSpec(Dg, H, 1).init(g).to(dev)
        slabv = torch.empty(ns, pv17.numel(), device=dev)
        fv = lambda: mlp_grad(GradHead.VALUE_MSE, pv17, Xv, 1, H, ret=ret, grad_slab=slabv, loss_slab=ls)  # noqa
        res["value_grad_d17_us"] = timeit(fv, a.iters)
        if a.stamps:
            run_stamps(fv, ns, 0, "value_d17", B)
    if a.which in ("fwd", "all"):
        out = {"v": torch.empty(B, device=dev)}
        us = timeit(lambda: mlp_forward(FwdMode.VALUE, pv, X, 1, H, out=out), a.iters)
        res["value_fwd_us"] = us
        res["value_fwd_TFLOPs"] = 2 * (D * H + H * H + H) * B / us / 1e6
        old = hip().set_value_fwd_mode(0)  # the fp32-MFMA forward, for comparison
        res["value_fwd_fp32mfma_us"] = timeit(lambda: mlp_forward(FwdMode.VALUE, pv, X, 1, H, out=out), a.iters)
        hip().set_value_fwd_mode(old)
    if a.which in ("adam", "all"):
        ns = hip().mlp_grad_slabs(B)
        slab = torch.randn(ns, pv.numel(), device=dev) * 1e-3
        m = torch.zeros_like(pv)
        v = torch.zeros_like(pv)
        step = torch.zeros(1, dtype=torch.int32, device=dev)
        tk = torch.zeros(1, dtype=torch.int32, device=dev)
        p2 = pv.clone()
        res["adam_us"] = timeit(lambda: adam_step(p2, m, v, step, tk, 1e-3, slab=slab), a.iters)
    if a.which in ("rslab", "all"):
        ns = hip().mlp_grad_slabs(B)
        slab = torch.randn(ns, pv.numel(), device=dev)
        out = torch.empty(pv.numel(), device=dev)
        res["reduce_slabs_us"] = timeit(lambda: reduce_slabs(slab, 1.0, out=out), a.iters)
    if a.which in ("scan", "all"):
        T, N = 64, B // 64
        rew = torch.rand(T, N, device=dev)
        done = (torch.rand(T, N, device=dev) < 0.05).float()
        val = torch.rand(T + 1, N, device=dev)
        advb = torch.empty(T, N, device=dev)
        retb = torch.empty(T, N, device=dev)
        res["scan_us"] = timeit(lambda: gae_scan_tm(rew, done, val, 0.99, 0.95, adv=advb, ret=retb), a.iters)
    if a.which in ("rollout", "all"):
        h = hip()
        T, N = 64, B // 64
        st = torch.zeros(N, 4, device=dev)
        el = torch.zeros(N, dtype=torch.int32, device=dev)
        er = torch.zeros(N, device=dev)
        obs = torch.empty(T + 1, N, 4, device=dev)
        ac = torch.empty(T, N, dtype=torch.int32, device=dev)
        lp = torch.empty(T, N, device=dev)
        rw = torch.empty(T, N, device=dev)
        dn = torch.empty(T, N, device=dev)
        es = torch.empty(h.rollout_grid(N), 8, device=dev)
        us = timeit(lambda: h.rollout(0, pp, H, st, el, er, obs, ac, lp, rw, dn, None, es, 1, 0, False, 500), a.iters)
        res["rollout_us"] = us
        res["rollout_Msteps_per_s"] = T * N / us
    print(json.dumps({k: round(v, 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()
