"""Micro-benchmark of the fc GEMMs (csrc/kernels/fc.hip) at the Pong A2C shapes, interleaved
A/B rounds in one process (HIP events): forward partials (2,048 x 512 x 3,136, split-K)
and the masked data gradient (10,240 x 3,136 x 512), for each RRL_FC_STAGES variant,
against the gemm_bf16.h kernels they replace.  One JSON line per (kernel, variant)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from relayrl_prototype_amd.models.nature_cnn import FC_IN, HIDDEN  # noqa: E402
from relayrl_prototype_amd.ops import hip  # noqa: E402


def timeit(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    h = hip()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    Mf, Mb = 2048, 10240
    a3 = torch.randn(Mb * FC_IN, device=dev, generator=g).relu().bfloat16()
    w = (torch.randn(HIDDEN * FC_IN, device=dev, generator=g) * 0.02).bfloat16()
    wt = torch.empty_like(w)
    h.transpose_bf16(w, wt, HIDDEN, FC_IN)
    dh = torch.randn(Mb * HIDDEN, device=dev, generator=g).bfloat16()
    b = torch.randn(HIDDEN, device=dev, generator=g)
    part = torch.empty(8 * Mf * HIDDEN, device=dev)
    hid = torch.empty(Mf * HIDDEN, dtype=torch.bfloat16, device=dev)
    da3 = torch.empty(Mb * FC_IN, dtype=torch.bfloat16, device=dev)
    work = torch.empty(16 * Mf * HIDDEN, device=dev)
    wpart = torch.empty(8 * HIDDEN * FC_IN, device=dev)
    Mx = 4 * Mb  # the 8192-env update (40,960 rows): outputs past the Infinity Cache
    partx = torch.empty(2 * 4 * Mf * HIDDEN, device=dev)
    a3x = torch.randn(Mx * FC_IN, device=dev, generator=g).relu().bfloat16()
    dhx = torch.randn(Mx * HIDDEN, device=dev, generator=g).bfloat16()
    da3x = torch.empty(Mx * FC_IN, dtype=torch.bfloat16, device=dev)

    def direct(fn):
        def run():
            os.environ["RRL_FC_DIRECT_EPI"] = "1"
            try:
                fn()
            finally:
                os.environ["RRL_FC_DIRECT_EPI"] = "0"  # forced staged for the other cases
        return run

    os.environ["RRL_FC_DIRECT_EPI"] = "0"
    cases = {
        "fwd_part_s4": lambda: h.fc_nt_part(a3, w, part, Mf, HIDDEN, FC_IN, 4),
        "fwd_part_s8": lambda: h.fc_nt_part(a3, w, part, Mf, HIDDEN, FC_IN, 8),
        "fwd8k_part_s2": lambda: h.fc_nt_part(a3x, w, partx, 4 * Mf, HIDDEN, FC_IN, 2),
        "fwd_old_gemm_bias_act": lambda: h.conv_fwd(a3[:Mf * FC_IN], w, b, hid, Mf, 1, 1, FC_IN, 1, 1, 1, HIDDEN,
                                                    True, work),
        "dgrad_mask": lambda: h.fc_nt_mask(dh, wt, a3, da3, Mb, FC_IN, HIDDEN),
        "dgrad_old": lambda: h.gemm_dgrad(dh, w, a3, da3, Mb, HIDDEN, FC_IN),
        "dgrad_mask_direct": direct(lambda: h.fc_nt_mask(dh, wt, a3, da3, Mb, FC_IN, HIDDEN)),
        "dgrad40k_mask": lambda: h.fc_nt_mask(dhx, wt, a3x, da3x, Mx, FC_IN, HIDDEN),
        "dgrad40k_mask_direct": direct(lambda: h.fc_nt_mask(dhx, wt, a3x, da3x, Mx, FC_IN, HIDDEN)),
        "wgrad_tn_s2": lambda: h.fc_tn_part(dh, a3, wpart, Mb, HIDDEN, FC_IN, 2),
        "wgrad_tn_s5": lambda: h.fc_tn_part(dh, a3, wpart, Mb, HIDDEN, FC_IN, 5),
        "wgrad_tn_s8": lambda: h.fc_tn_part(dh, a3, wpart, Mb, HIDDEN, FC_IN, 8),
        "wgrad40k_tn_s5": lambda: h.fc_tn_part(dhx, a3x, wpart, Mx, HIDDEN, FC_IN, 5),
        "wgrad_old_s2": lambda: h.conv_wgrad(dh, a3, wpart, 2, Mb, 1, 1, FC_IN, 1, 1, 1, HIDDEN),
    }
    # "b" in a variant = the persistent 256 x 128 kernels (RRL_FC_BIG=1), else the 128 x 128 ones
    variants = os.environ.get("FC_VARIANTS", "422,b").split(",")
    only = [c for c in os.environ.get("FC_CASES", "").split(",") if c]
    if only:
        cases = {k: v for k, v in cases.items() if k in only}
    res = {}
    for _ in range(int(os.environ.get("FC_ROUNDS", "5"))):
        for v in variants:
            os.environ["RRL_FC_STAGES"] = v.replace("m", "").replace("b", "").replace("p", "")
            os.environ["RRL_FC_MFAST"] = "1" if "m" in v else "0"
            os.environ["RRL_FC_BIG"] = "1" if "b" in v else "0"
            os.environ["RRL_FC_SETPRIO"] = "1" if "p" in v else "0"
            for k, fn in cases.items():
                if "old" in k and v != variants[0]:
                    continue
                res.setdefault((k, v if "old" not in k else "-"), []).append(timeit(fn))
    for (k, v), ts in res.items():
        print(json.dumps({"probe": "fc_kbench", "case": k, "stages": v, "median_us": round(statistics.median(ts), 2),
                          "min_us": round(min(ts), 2)}))


if __name__ == "__main__":
    main()
