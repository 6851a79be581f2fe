#!/usr/bin/env python3
"""One-rank RCCL probe: communicator init, all_reduce / broadcast / all_gather on HBM tensors,
and whether an all_reduce can be captured into a hipGraph (the multi-rank value loop's open
question, docs/PERF_NOTES.md).  Prints one JSON line."""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    t = torch.arange(17281, device="cuda", dtype=torch.float32)
    ref = t.clone()
    dist.all_reduce(t)
    dist.broadcast(t, 0)
    lst = [torch.empty_like(t)]
    dist.all_gather(lst, t)
    torch.cuda.synchronize()
    out["collectives_ok"] = bool(torch.equal(t, ref) and torch.equal(lst[0], ref))
    # latency of a 69 KB all_reduce (one rank: the RCCL launch + kernel floor)
    for _ in range(5):
        dist.all_reduce(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        dist.all_reduce(t)
    torch.cuda.synchronize()
    out["all_reduce_69KB_us"] = (time.perf_counter() - t0) / 200 * 1e6
    # hipGraph capture of scale + all_reduce, replayed
    try:
        x = torch.ones(17281, device="cuda")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            x.mul_(2.0)
            dist.all_reduce(x)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            x.mul_(2.0)
            dist.all_reduce(x)
        x.fill_(1.0)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        out["graph_capture_ok"] = bool(torch.all(x == 8.0).item())
    except Exception as e:  # report, do not hide
        out["graph_capture_ok"] = False
        out["graph_capture_error"] = repr(e)[:300]
    dist.destroy_process_group()
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
