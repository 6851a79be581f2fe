#!/usr/bin/env python3
"""Micro-benchmark of the pixel-model conv kernels at the Pong A2C shapes (2,048-frame
rollout forward, 10,240-frame update backward): per-launch microseconds from HIP events.

    python tools/cnn_kbench.py [--which fwd,bwd3,dgrad2,wgrad1] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="fwd,fwd_layers,bwd3,bwd3_layers,bwd2,dgrad2,wgrad1,wgrad1_8")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=1, help="repeat the list, alternating its order; median per kernel")
    ap.add_argument("--frames", type=int, default=2048)
    ap.add_argument("--bwd-frames", type=int, default=10240)
    a = ap.parse_args()
    from relayrl_prototype_amd.models.nature_cnn import CONVS, FC_IN, S2D, CNNSpec
    from relayrl_prototype_amd.ops import hip

    h = hip()
    dev = torch.device("cuda", 0)
    spec = CNNSpec()
    o = spec.offsets()
    p = spec.init(1).to(dev)
    sh = p.bfloat16()
    Nf, Nb = a.frames, a.bwd_frames
    N = max(Nf, Nb)
    x = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, device=dev)
    a1 = torch.empty(N * 400 * 32, dtype=torch.bfloat16, device=dev)
    a2 = torch.empty(N * 81 * 64, dtype=torch.bfloat16, device=dev)
    a3 = torch.empty(N * FC_IN, dtype=torch.bfloat16, device=dev)
    da3 = (torch.randn(N * FC_IN, device=dev) * 0.01).bfloat16()
    da2 = torch.empty_like(a2)
    da1 = torch.empty_like(a1)
    cus = int(h.device_cus())
    part = torch.empty(cus * 64 * 576 * 4, device=dev)
    bpart = torch.empty(cus * 512 * 4, device=dev)
    W = {i: (sh[o[f"w{i}"]:o[f"b{i}"]], p[o[f"b{i}"]:o[f"b{i}"] + CONVS[i - 1].cout]) for i in (1, 2, 3)}
    h.conv_stack_fwd(x, *W[1], *W[2], *W[3], a1, a2, a3, N)  # activations for the backward shapes

    def fwd():
        h.conv_stack_fwd(x, *W[1], *W[2], *W[3], a1, a2, a3, Nf)

    def probe(k, grid=0):
        return lambda: h.conv_stack_fwd(x, *W[1], *W[2], *W[3], a1, a2, a3, Nf, probe=k, grid=grid)

    def fwd_layers():
        src = x
        for i, (L, y) in enumerate(zip((S2D,) + CONVS[1:], (a1, a2, a3)), 1):
            h.conv_fwd(src, *W[i], y, Nf, L.hin, L.hin, L.cin, L.k, L.k, L.s, L.cout, True)
            src = y

    def bwd3():
        h.conv3_bwd(da3, W[3][0], a2, da2, part, bpart, Nb, min(Nb, cus))

    def bwd3_16():
        h.conv3_bwd(da3, W[3][0], a2, da2, part, bpart, Nb, min(Nb, cus), variant=1)

    def bwd3_layers():
        L = CONVS[2]
        h.conv_dgrad(da3, W[3][0], a2, da2, Nb, L.hin, L.hin, L.cin, L.k, L.k, L.s, L.cout)

    def dgrad2():
        L = CONVS[1]
        h.conv_dgrad(da2, W[2][0], a1, da1, Nb, L.hin, L.hin, L.cin, L.k, L.k, L.s, L.cout)

    fns = {}
    fns["wgrad1_8"] = lambda: h.conv1_wgrad8(x[:Nb], da1, part, bpart, Nb, min(Nb, cus))
    # frame ring (envs/pong.FrameRing): R = 9 slots x Nf envs; row n = t Nf + e of a T-step rollout
    # reads frames t .. t + 3 of env e (the rollout's sharing pattern, 3 of 4 frames shared by rows
    # t and t + 1 of one env)
    R = 9
    frames = torch.randint(0, 256, (R * Nf * 7056,), dtype=torch.uint8, device=dev)
    rows = torch.arange(N, device=dev)
    e, t = rows % Nf, rows // Nf
    fidx = torch.stack([((t + f) % R) * Nf + e for f in range(4)], 1).int().contiguous()
    Tb = Nb // Nf if Nb % Nf == 0 else 0
    fns["fwd16_ring"] = lambda: h.conv_stack_fwd(None, *W[1], *W[2], *W[3], a1, a2, a3, Nf, frames=frames,
                                                 fidx=fidx[:Nf])
    fns["fwd16_ring16"] = lambda: h.conv_stack_fwd(None, *W[1], *W[2], *W[3], a1, a2, a3, Nf, probe=192,
                                                   frames=frames, fidx=fidx[:Nf])
    fns["fwd16_ring_wide"] = lambda: h.conv_stack_fwd(None, *W[1], *W[2], *W[3], a1, a2, a3, Nf, probe=320,
                                                      frames=frames, fidx=fidx[:Nf])
    fns["wgrad1_8_ring"] = lambda: h.conv1_wgrad8(None, da1, part, bpart, Nb, min(Nb, cus), frames=frames,
                                                  fidx=fidx[:Nb])
    fns["wgrad1_8_ring_em"] = lambda: h.conv1_wgrad8(None, da1, part, bpart, Nb, min(Nb, cus), frames=frames,
                                                     fidx=fidx[:Nb], env_major_T=Tb)

    def wgrad1_8_sp():  # the s_setprio form (RRL_CNN_WGRAD1_SETPRIO, read per call)
        os.environ["RRL_CNN_WGRAD1_SETPRIO"] = "1"
        try:
            h.conv1_wgrad8(x[:Nb], da1, part, bpart, Nb, min(Nb, cus))
        finally:
            os.environ["RRL_CNN_WGRAD1_SETPRIO"] = "0"
    fns["wgrad1_8_sp"] = wgrad1_8_sp
    fns["fwd16_sp"] = probe(68)
    fns["fwd16_prio2"] = probe(65)  # static priority: the conv2 role
    fns["fwd16_prio3"] = probe(72)  # the conv3 role
    fns["fwd16_prio23"] = probe(73)
    fns["wgrad1"] = lambda: h.conv_wgrad(da1, x[:Nb], part, 256, Nb, 21, 21, 64, 2, 2, 1, 32, bpart)
    fns.update({"p_nomfma": probe(1), "p_nostore": probe(2), "p_nostore_nomfma": probe(3), "p_hotframe": probe(4),
           "p_all": probe(7), "fwd_c1split": probe(8), "fwd_g128": probe(0, 128), "fwd_phase_a1": probe(16), "fwd_c3_grid": probe(32), "fwd_phase_a1_c3_grid": probe(48), "fwd_g512": probe(0, 512), "fwd8": probe(128), "fwd16": probe(64), "fwd16_phase": probe(80), "fwd16_grid3": probe(96), "fwd16_both": probe(112), "fwd": fwd, "fwd_layers": fwd_layers, "bwd3": bwd3, "bwd3_16": bwd3_16, "bwd3_layers": bwd3_layers, "dgrad2": dgrad2})
    if hasattr(h, "conv2_bwd"):
        def bwd2():
            h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus))

        def bwd2_staged():
            h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=1)
        fns["bwd2"] = bwd2
        fns["bwd2_staged"] = bwd2_staged
        fns["bwd2_16"] = lambda: h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=3)
        fns["bwd2_grid12"] = lambda: h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=2)
        # wave priority (s_setprio): 4 = around each MFMA cluster, 5 = waves 4-7 raised for the kernel
        fns["bwd2_sp1"] = lambda: h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=4)
        fns["bwd2_sp2"] = lambda: h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=5)
        fns["bwd2_sp_w"] = lambda: h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=6)
        fns["bwd2_sp_d"] = lambda: h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=7)
        fns["bwd2_st16"] = lambda: h.conv2_bwd(da2, W[2][0], a1, da1, part, bpart, Nb, min(Nb, cus), staged=8)
    # conv3 backward wave priority: bwd3 = the shipped s_setprio-cluster form, bwd3_sp0 = without
    fns["bwd3_sp0"] = lambda: h.conv3_bwd(da3, W[3][0], a2, da2, part, bpart, Nb, min(Nb, cus), variant=2)
    fns["bwd3_sp2"] = lambda: h.conv3_bwd(da3, W[3][0], a2, da2, part, bpart, Nb, min(Nb, cus), variant=3)
    fns["bwd3_sp_w"] = lambda: h.conv3_bwd(da3, W[3][0], a2, da2, part, bpart, Nb, min(Nb, cus), variant=4)
    fns["bwd3_sp_d"] = lambda: h.conv3_bwd(da3, W[3][0], a2, da2, part, bpart, Nb, min(Nb, cus), variant=5)
    fns["bwd3_16_sp"] = lambda: h.conv3_bwd(da3, W[3][0], a2, da2, part, bpart, Nb, min(Nb, cus), variant=6)

    # --rounds R: the list R times, every other round in reverse order (the first kernel timed
    # in a process reads slow), median per kernel
    names = a.which.split(",")
    times = {n: [] for n in names}
    for r in range(a.rounds):
        for name in (names if r % 2 == 0 else names[::-1]):
            f = fns[name]
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    out = {n: round(sorted(t)[len(t) // 2], 1) for n, t in times.items()}
    print(json.dumps({"bench": "cnn_kbench", "frames_fwd": Nf, "frames_bwd": Nb, "us_per_launch": out}), flush=True)


if __name__ == "__main__":
    main()
