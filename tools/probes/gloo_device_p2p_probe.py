"""Does gloo P2P on a device tensor wait for the kernels queued before it?

Two gloo ranks share cuda:0.  Rank 0 queues ~tens of ms of matmuls, then a fill of the send
buffer with the round number, and posts the isend straight away (``--fence 0``) or after
synchronising its stream (``--fence 1``, what ``Comm.gather_to`` / ``ActorLearner`` do for a
non-RCCL backend).  Rank 1 counts rounds whose received buffer is not the round number
everywhere.  Prints one JSON line from rank 1.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/probes/gloo_device_p2p_probe.py --fence 0
"""
import argparse
import json
import os

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fence", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--op", choices=("p2p", "all_reduce", "broadcast"), default="p2p",
                    help="all_reduce / broadcast: the gloo collective on the device buffer instead of send / recv")
    ap.add_argument("--via", choices=("dist", "comm"), default="dist",
                    help="comm: the transfer is Comm.gather_to (its own fence for non-RCCL backends)")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    comm = None
    if a.via == "comm":
        from relayrl_prototype_amd.parallel.comm import Comm

        comm = Comm()
    torch.cuda.set_device(0)
    buf = torch.zeros(a.n, device="cuda")
    m = torch.randn(2048, 2048, device="cuda")
    torn = 0
    for r in range(1, a.rounds + 1):
        dist.barrier()
        if a.op != "p2p":  # every rank writes its buffer late, then the collective runs at once
            x = m
            for _ in range(40):
                x = torch.tanh(x @ m)
            buf.fill_(float(r))
            buf[:1].add_(x[:1, 0] * 0)
            if a.fence:
                torch.cuda.current_stream().synchronize()
            if a.op == "all_reduce":
                dist.all_reduce(buf)
                want = 2.0 * r
            else:
                if rank == 1:
                    buf.fill_(-1.0)
                dist.broadcast(buf, 0)
                want = float(r)
            torch.cuda.synchronize()
            if rank == 1 and not bool((buf == want).all()):
                torn += 1
            continue
        if rank == 0:
            x = m
            for _ in range(40):  # keep the stream busy so the fill below runs late
                x = torch.tanh(x @ m)
            buf.fill_(float(r))
            buf[:1].add_(x[:1, 0] * 0)  # the fill stays after the matmuls in stream order
            if a.fence:
                torch.cuda.current_stream().synchronize()
            if comm is not None:
                comm.gather_to(buf, 1)
            else:
                dist.send(buf, 1)
        else:
            if comm is not None:
                own = torch.zeros_like(buf)
                comm.gather_to(own, 1, out=[buf, own])
            else:
                dist.recv(buf, 0)
            torch.cuda.synchronize()
            if not bool((buf == float(r)).all()):
                torn += 1
    if rank == 1:
        print(json.dumps({"op": a.op, "via": a.via, "fence": a.fence, "rounds": a.rounds, "stale_or_torn_rounds": torn,
                          "backend": "gloo", "device": torch.cuda.get_device_name(0)}), flush=True)
    dist.destroy_process_group()
    os._exit(0)


if __name__ == "__main__":
    main()
