"""Per-iteration cost of the small-batch value loop behind the reference-hyperparameter
time-to-threshold (512 envs x 16 steps = 8,192 rows, 80 value iterations per epoch), and the
"fewer, fatter slabs" lever measured directly: the grid of the value-gradient kernel is capped
with ``set_cu_limit`` (64-row slabs, one per workgroup, so the cap IS the slab count), and the
captured loop, the gradient kernel alone and the reduce+Adam kernel alone are timed per cap.

    python tools/ttt_levers_probe.py [--B 8192] [--iters 80] [--caps 0,96,64,32]

One JSON line per cap: loop / grad / adam microseconds per iteration and the slab count
(adam_us: every update pays the arrival ticket; adam_loop_form_us: one ticket per loop, as
ValueLoop runs it since round 4).
(The stamp build -- ``tools/kbench.py grad --B 8192 --stamps`` -- gives the prologue /
per-slab / epilogue split of the gradient kernel that prices the split-image lever.)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from relayrl_prototype_amd.algorithms.core import FlatNet, ValueLoop  # noqa: E402
from relayrl_prototype_amd.ops import GradHead, MLPSpec, adam_step, grad_slabs, mlp_grad  # noqa: E402
from relayrl_prototype_amd.ops import hip  # noqa: E402


def graph_time(fn, reps=20):
    """Microseconds per replay of a captured ``fn``."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8192)
    ap.add_argument("--D", type=int, default=4)
    ap.add_argument("--iters", type=int, default=80)
    ap.add_argument("--caps", default="0,96,64,32")
    a = ap.parse_args()
    dev = torch.device("cuda")
    h = hip()
    torch.manual_seed(0)
    spec = MLPSpec(a.D, 128, 1)
    obs = torch.randn(a.B, a.D, device=dev)
    ret = torch.randn(a.B, device=dev) * 10
    inv_B = 1.0 / a.B
    for cap in [int(c) for c in a.caps.split(",")]:
        old = h.set_cu_limit(cap)
        try:
            ns = grad_slabs(a.B, dev)
            net = FlatNet(spec, 1e-3, dev, generator=torch.Generator().manual_seed(1))
            loop = ValueLoop(net, None, use_graph=True)
            loop.run(obs, ret, a.iters, inv_B)  # capture
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            reps = 10
            for _ in range(reps):
                loop.run(obs, ret, a.iters, inv_B)
            e1.record()
            torch.cuda.synchronize()
            loop_us = e0.elapsed_time(e1) / reps / a.iters * 1e3
            slab = torch.empty(ns, spec.P, device=dev)
            ls = torch.empty(ns, 8, device=dev)

            def grads():
                for _ in range(a.iters):
                    mlp_grad(GradHead.VALUE_MSE, net.params, obs, 1, 128, ret=ret, inv_B=inv_B, grad_slab=slab,
                             loss_slab=ls)

            def adams():
                for _ in range(a.iters):
                    adam_step(net.params, net.m, net.v, net.step, net.ticket, 1e-9, slab=slab)

            def adams_loop():  # the loop form of the step counter: one arrival ticket per loop
                for k in range(a.iters):
                    adam_step(net.params, net.m, net.v, net.step, net.ticket, 1e-9, slab=slab, step_add=k,
                              step_inc=a.iters if k == a.iters - 1 else 0)

            grad_us = graph_time(grads) / a.iters
            adam_us = graph_time(adams) / a.iters
            adam_loop_us = graph_time(adams_loop) / a.iters
            print(json.dumps({"B": a.B, "cu_cap": cap, "slabs": ns, "loop_us_per_iter": round(loop_us, 2),
                              "grad_us": round(grad_us, 2), "adam_us": round(adam_us, 2),
                              "adam_loop_form_us": round(adam_loop_us, 2),
                              "epoch_value_loop_ms": round(loop_us * a.iters / 1e3, 3)}), flush=True)
        finally:
            h.set_cu_limit(old)


if __name__ == "__main__":
    main()
