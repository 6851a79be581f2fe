"""Multi-process data-parallel paths on CPU with gloo (world_size 2).

The same code runs one process per MI355X with RCCL; here gloo + the PyTorch oracle ops
validate the collective logic: gradient all-reduce (C8), weight broadcast (C2),
rollout fan-in gather (C1) and global advantage statistics.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from relayrl_prototype_amd.parallel.comm import init_distributed

    return init_distributed(backend="gloo")


def _worker_grad_allreduce(rank, world, port, q):
    try:
        comm = _init(rank, world, port)
        from relayrl_prototype_amd.algorithms.core import FlatNet
        from relayrl_prototype_amd.ops import MLPSpec
        from relayrl_prototype_amd.ops import reference as ref

        spec = MLPSpec(3, 64, 2)
        net = FlatNet(spec, 1e-2, "cpu", torch.Generator().manual_seed(0))
        g = torch.Generator().manual_seed(100 + rank)
        slab = torch.randn(2, spec.P, generator=g)
        net.apply(slab, comm)
        # oracle: Adam on the rank-sum of all slabs
        all_slabs = [torch.randn(2, spec.P, generator=torch.Generator().manual_seed(100 + r)) for r in range(world)]
        p = spec.init(torch.Generator().manual_seed(0))
        m = torch.zeros_like(p)
        v = torch.zeros_like(p)
        ref.adam_ref(p, m, v, sum(s.sum(0) for s in all_slabs), 1, 1e-2)
        q.put((rank, torch.allclose(net.params, p, atol=1e-6), net.params.sum().item()))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None))


def _worker_trainer(rank, world, port, q):
    try:
        comm = _init(rank, world, port)
        from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

        cfg = HostTrainerConfig(env="CartPole-v1", num_envs=16, rollout_len=16, algo="ppo", hidden=64,
                                train_vf_iters=2, train_pi_iters=2, num_threads=1, seed=3)
        tr = HostVecTrainer(cfg, comm, device="cpu")
        for _ in range(2):
            tr.train_epoch()
        m = tr.metrics()
        gathered = [torch.zeros_like(tr.learner.pi.params) for _ in range(world)]
        dist.all_gather(gathered, tr.learner.pi.params)
        same = all(torch.equal(gathered[0], x) for x in gathered)
        # rollout fan-in: gather each rank's rewards on rank 0 over point-to-point links
        out = [torch.zeros_like(tr.d_rew) for _ in range(world)] if rank == 0 else None
        comm.gather_to(tr.d_rew.contiguous(), 0, out)
        fanin_ok = True if rank != 0 else all(o.shape == tr.d_rew.shape for o in out)
        # weight broadcast from the learner rank
        w = tr.learner.pi.params.clone() if rank == 0 else torch.zeros_like(tr.learner.pi.params)
        comm.broadcast_(w, 0)
        q.put((rank, same and fanin_ok and torch.equal(w, gathered[0]), m["EnvSteps"]))
        dist.destroy_process_group()
    except Exception as e:
        import traceback

        q.put((rank, traceback.format_exc(), None))


def _run(fn, world=2):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    return sorted(res, key=lambda r: r[0])


def test_dp_gradient_allreduce_matches_oracle():
    res = _run(_worker_grad_allreduce)
    for rank, ok, s in res:
        assert ok is True, (rank, ok)
    assert res[0][2] == res[1][2]


def test_dp_host_trainer_ranks_stay_in_sync():
    res = _run(_worker_trainer)
    for rank, ok, steps in res:
        assert ok is True, (rank, ok)
        assert steps == 2 * 16 * 16 * 2


def _al_worker(rank, world, port, q, lag=0, learners=0, learner_acts=True, steps=3, verify=True, algo="reinforce"):
    try:
        comm = _init(rank, world, port)
        from relayrl_prototype_amd.runtime.actor_learner import ActorLearner, ActorLearnerConfig

        cfg = ActorLearnerConfig(env="CartPole-v1", num_envs=8, rollout_len=16, algo=algo, hidden=64,
                                 train_vf_iters=2, train_pi_iters=2, num_threads=1, seed=5, max_lag=lag,
                                 learner_ranks=learners, learner_acts=learner_acts, verify_versions=verify)
        al = ActorLearner(cfg, comm, device="cpu")
        versions = []
        for _ in range(steps):
            al.step()
            if al.is_learner:
                versions.append([int(x) for x in al.b_hdr[:, 7].tolist()])
        al.finish()
        m = al.metrics()
        w = al.wbuf.clone()
        gathered = [torch.zeros_like(w) for _ in range(world)]
        dist.all_gather(gathered, w)
        same = all(torch.equal(gathered[0], x) for x in gathered)
        q.put((rank, same, m.get("EnvSteps"), m.get("ActorSeqs"), versions, w.numpy().copy(), m.get("Episodes")))
        dist.destroy_process_group()
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc(), None, None, None, None, None))


def _worker_actor_learner(rank, world, port, q):
    # classic topology: rank 0 learns only, ranks 1, 2 act
    _al_worker(rank, world, port, q, lag=0, learners=1, learner_acts=False)


def _worker_actor_learner_lag(rank, world, port, q):
    _al_worker(rank, world, port, q, lag=1, learners=1, learner_acts=False)


@pytest.mark.parametrize("fn", [_worker_actor_learner, _worker_actor_learner_lag])
def test_actor_learner_gloo(fn):
    res = _run(fn, world=3)
    for r in res:
        assert r[1] is True, (r[0], r[1])
    assert res[0][2] == 3 * 16 * 8 * 2  # two actors x 3 rollouts
    assert res[0][3] == [3.0, 3.0]       # per-actor heartbeat sequence numbers
    lag = 1 if fn is _worker_actor_learner_lag else 0
    # version of the weights each rollout used: exactly k (sync) or max(k-1, 0) (lag 1);
    # verify_versions also matched every rollout's weight checksum against that version
    for k, vs in enumerate(res[0][4]):
        assert vs == [max(k - lag, 0)] * 2, (k, vs)


def _worker_group_l2(rank, world, port, q):
    # W = 4, L = 2: every rank acts, ranks 0 and 1 learn on two actor blocks each
    _al_worker(rank, world, port, q, lag=0, learners=2, learner_acts=True, steps=2, algo="ppo")


def _worker_group_dp(rank, world, port, q):
    # oracle: plain data parallel (every rank learns its own rollout)
    _al_worker(rank, world, port, q, lag=0, learners=4, learner_acts=True, steps=2, algo="ppo")


def test_learner_group_matches_data_parallel_oracle():
    g = _run(_worker_group_l2, world=4)
    o = _run(_worker_group_dp, world=4)
    for r in g + o:
        assert r[1] is True, (r[0], r[1])
    assert g[0][2] == o[0][2] == 2 * 16 * 8 * 4
    assert g[0][6] == o[0][6]  # identical episode statistics (same rollouts)
    # same weights up to the summation order of the gradient (2 shards x 2 blocks vs 4 x 1)
    torch.testing.assert_close(torch.from_numpy(g[0][5]), torch.from_numpy(o[0][5]), rtol=1e-5, atol=1e-6)


def _worker_group_lag(rank, world, port, q):
    # W = 4, L = 2, learners only learn: actors 2, 3 feed shards 0, 1 with lag-1 weights
    _al_worker(rank, world, port, q, lag=1, learners=2, learner_acts=False, steps=4)


def test_learner_group_lag1_versions_never_torn():
    res = _run(_worker_group_lag, world=4)
    for r in res:
        assert r[1] is True, (r[0], r[1])
    for lr in (0, 1):
        assert [v[0] for v in res[lr][4]] == [0, 0, 1, 2]


def _worker_stall(rank, world, port, q):
    import time

    try:
        comm = _init(rank, world, port)
        from relayrl_prototype_amd.runtime.actor_learner import ActorLearner, ActorLearnerConfig

        cfg = ActorLearnerConfig(env="CartPole-v1", num_envs=8, rollout_len=16, hidden=64, train_vf_iters=2,
                                 num_threads=1, seed=5, learner_ranks=1, learner_acts=False, stall_timeout_s=3.0)
        def report(msg):  # flush the queue's feeder thread: the watchdog exits right after
            q.put((rank, "stall", msg))
            q.close()
            q.join_thread()

        al = ActorLearner(cfg, comm, device="cpu", on_stall=report)
        for k in range(4):
            if rank == 2 and k == 2:
                time.sleep(60)  # a hung actor: no rollout, no heartbeat
            al.step()
        q.put((rank, "done", None))
    except Exception as e:
        q.put((rank, "error", repr(e)))


def test_stalled_actor_is_named_and_learner_exits_for_restart():
    """Actor 2 hangs before its third rollout: the learner's step watchdog names it (with
    its last heartbeat) within the per-epoch budget -- not the 10-minute collective timeout
    -- and exits with EXIT_STALL so torchrun restarts the group."""
    import time

    from relayrl_prototype_amd.utils.watchdog import EXIT_STALL

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_stall, args=(r, 3, port, q)) for r in range(3)]
    t0 = time.time()
    for p in ps:
        p.start()
    try:
        msgs = []
        while time.time() - t0 < 90:
            try:
                msgs.append(q.get(timeout=1))
            except Exception:
                pass
            if any(m[0] == 0 and m[1] == "stall" for m in msgs):
                break
        stall = [m for m in msgs if m[0] == 0 and m[1] == "stall"]
        assert stall, msgs
        assert "actor(s) [2]" in stall[0][2] and "rollout 2" in stall[0][2], stall[0][2]
        assert time.time() - t0 < 60
        ps[0].join(timeout=20)
        assert ps[0].exitcode == EXIT_STALL
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
            p.join(timeout=10)
