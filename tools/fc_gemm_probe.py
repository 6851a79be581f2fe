#!/usr/bin/env python3
"""Pong A2C fc layer GEMMs: the hand-written bf16 MFMA path (cnn.hip) vs hipBLASLt through
torch, per call (HIP events, median of 50)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def t_ms(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from relayrl_prototype_amd.ops import hip

    h = hip()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    K, N = 3136, 512
    for M in (2048, 10240):
        a3 = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.02).to(bf)
        b = torch.randn(N, device=dev)
        hid = torch.empty(M, N, dtype=bf, device=dev)
        part = torch.empty(8 * M * N, device=dev)
        ours = t_ms(lambda: h.conv_fwd(a3.view(-1), w.view(-1), b, hid.view(-1), M, 1, 1, K, 1, 1, 1, N, True, part))
        bb = b.to(bf)
        lib = t_ms(lambda: torch.relu_(torch.addmm(bb, a3, w.t())))
        lib_act = None
        try:
            lib_act = t_ms(lambda: torch._addmm_activation(bb, a3, w.t(), use_gelu=False))
        except Exception as e:  # noqa: BLE001
            lib_act = repr(e)[:80]
        dh = torch.randn(M, N, device=dev).to(bf)
        wg = t_ms(lambda: torch.mm(dh.t(), a3))          # fc weight gradient [N, K]
        dg = t_ms(lambda: torch.mm(dh, w))               # fc data gradient [M, K] (before the ReLU mask)
        print(json.dumps({"M": M, "N": N, "K": K, "fwd_ours_ms": ours, "fwd_hipblaslt_addmm_relu_ms": lib,
                          "fwd_hipblaslt_fused_act_ms": lib_act, "wgrad_hipblaslt_ms": wg, "dgrad_hipblaslt_ms": dg,
                          "gflop_fwd": 2 * M * N * K / 1e9}), flush=True)


if __name__ == "__main__":
    main()
