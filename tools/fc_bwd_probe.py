#!/usr/bin/env python3
"""fc layer backward at the Pong update shape (10,240 rows, 3136 -> 512): our bf16 MFMA GEMMs
(split-K weight gradient + split sum; masked data gradient) against hipBLASLt through
torch.mm (fp32-output weight gradient; bf16 data gradient + a separate mask pass)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timeit(f, iters=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / iters, 1)


def main():
    from relayrl_prototype_amd.ops import hip

    h = hip()
    dev = torch.device("cuda", 0)
    B, F, K = 10240, 512, 3136
    dh = (torch.randn(B, F, device=dev) * 0.01).bfloat16()
    a3 = torch.relu(torch.randn(B, K, device=dev)).bfloat16()
    W = (torch.randn(F, K, device=dev) * 0.02).bfloat16()
    splits = int(h.gemm_splits(B, 32))
    part = torch.empty(splits * F * K, device=dev)
    gw = torch.empty(F * K, device=dev)
    da3 = torch.empty(B * K, dtype=torch.bfloat16, device=dev)
    out = {}

    def ours_wgrad():
        s = int(h.conv_wgrad(dh.reshape(-1), a3.reshape(-1), part, 32, B, 1, 1, K, 1, 1, 1, F, None))
        h.sum_splits(part, s, F * K, gw)

    out["ours_wgrad_us"] = timeit(ours_wgrad)
    out["blas_wgrad_fp32out_us"] = timeit(lambda: torch.mm(dh.t(), a3, out_dtype=torch.float32))
    out["ours_dgrad_masked_us"] = timeit(lambda: h.gemm_dgrad(dh.reshape(-1), W.reshape(-1), a3.reshape(-1),
                                                              da3, B, F, K))
    out["blas_dgrad_us"] = timeit(lambda: torch.mm(dh, W))
    out["blas_dgrad_plus_mask_us"] = timeit(lambda: torch.mm(dh, W).mul_(a3 > 0))
    ref = torch.mm(dh.t().float(), a3.float())
    ours_wgrad()
    out["ours_wgrad_relerr"] = float((gw.view(F, K) - ref).norm() / ref.norm())
    out["blas_wgrad_relerr"] = float((torch.mm(dh.t(), a3, out_dtype=torch.float32) - ref).norm() / ref.norm())
    print(json.dumps({"probe": "fc_bwd", "rows": B, **out}), flush=True)


if __name__ == "__main__":
    main()
