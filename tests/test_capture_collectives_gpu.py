"""whether a rank captures a new graph this epoch is a rank-local decision
(its own input buffers, agent rows folded on rank 0 only, a per-rank cache eviction), so the
eager warm-up before a capture must not issue collectives -- they would pair with another
rank's unrelated calls.  A recording comm on the multi-rank code path (``multi``, graph-safe)
shows every collective is issued INSIDE a capture (replayed by every rank's graph, same
sequence for any batch shape) and none by the warm-ups.  And a capture for
a new batch shape must not free the buffers an earlier graph replays into: alternating padded
(agent rows) and unpadded epochs with allocation churn in between equal the eager run, with
the value loss read from the replayed graph's own slabs."""
import numpy as np
import pytest
import torch

from relayrl_prototype_amd.parallel.comm import Comm

pytestmark = pytest.mark.gpu


class _RecComm(Comm):
    """The world > 1 code path on one process: collectives are recorded, not communicated."""

    def __init__(self):
        super().__init__(collectives=False)
        self.multi = True
        self.backend = "nccl"
        self.calls = []

    def all_reduce_sum_(self, t):
        if not self._muted:
            self.calls.append((int(t.numel()), torch.cuda.is_current_stream_capturing()))
        return t


def test_capture_warmups_issue_no_collectives(cuda):
    from relayrl_prototype_amd.algorithms.learner import PGLearner

    comm = _RecComm()
    lr = PGLearner("reinforce", 4, 2, 128, True, True, train_vf_iters=6, device=cuda, comm=comm, seed=1)
    P = lr.pi.P

    def batch(B, seed):
        g = torch.Generator(device="cpu").manual_seed(seed)
        obs = torch.randn(B, 4, generator=g).to(cuda)
        act = torch.randint(0, 2, (B,), generator=g, dtype=torch.int32).to(cuda)
        adv, ret = torch.randn(B, generator=g).to(cuda), torch.randn(B, generator=g).to(cuda)
        return obs, act, adv, ret, torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(B), device=cuda)])

    a = batch(4096, 0)
    b = batch(4096 + 512, 1)  # a padded agent-row batch: a new graph key on this rank only
    for k, (obs, act, adv, ret, st) in enumerate((a, a, b, a, b)):
        n0 = len(comm.calls)
        lr.optimize(obs, act=act, adv=adv, ret=ret, adv_stats=st)
        new = comm.calls[n0:]
        if k in (0, 2):  # a capture: exactly one gradient all-reduce per optimiser step, all captured
            assert len(new) == 1 + 6 and all(c for _, c in new), new
            assert {n for n, _ in new} == {P, lr.vf.P}
        else:  # a replay issues nothing from Python (the graph holds the collectives)
            assert new == []
    assert lr.graph_replays == 5


def test_alternating_padded_and_unpadded_graphs_keep_their_buffers(cuda, tmp_path):
    from relayrl_prototype_amd.runtime.engine import EngineAlgorithm, EngineSpec
    from relayrl_prototype_amd.types import TrajectoryColumns

    def episode(rng, n):
        obs = rng.normal(size=(n, 4)).astype(np.float32) * 0.1
        act = rng.integers(0, 2, size=(n, 1)).astype(np.int32)
        done = np.zeros(n, np.uint8)
        done[-1] = 1
        return TrajectoryColumns(obs, act, np.ones(n, np.float32), done, None, np.full(n, -0.69, np.float32),
                                 "agent-0", 0)

    res = {}
    for graphs in (False, True):
        rng = np.random.default_rng(0)
        churn_rng = torch.Generator(device="cpu").manual_seed(5)
        spec = EngineSpec("vec", "CartPole-v1", "reinforce", 1,
                          {"env": "CartPole-v1", "algo": "reinforce", "num_envs": 256, "rollout_len": 16,
                           "train_vf_iters": 5, "use_graphs": graphs, "seed": 3, "with_baseline": True})
        algo = EngineAlgorithm(spec, str(tmp_path / f"g{int(graphs)}"), device=cuda, log=False, agent_buf_size=512)
        losses, rows = [], []
        for ep in range(8):
            if ep % 2 == 0:  # uploads on even epochs only: padded / unpadded graphs alternate
                algo.receive_trajectory(episode(rng, 20 + 7 * ep))
            algo.train_model()
            rows.append(int(algo.trainer.rl.last_agent_rows))
            losses.append(algo.learner.summarize()["LossV"])
            # allocation churn: freed blocks of every size get reused if a graph's buffer was freed
            junk = [torch.randn(int(n), generator=churn_rng).to(cuda) for n in (4096, 65536, 1 << 20, 17000 * 64)]
            del junk
        torch.cuda.synchronize()
        res[graphs] = (algo.learner.pi.params.cpu(), algo.learner.vf.params.cpu(), rows, losses,
                       algo.learner.graph_replays)
    e, g = res[False], res[True]
    assert e[2] == g[2] and e[2][0] > 0 and e[2][1] == 0
    assert g[4] == 8
    np.testing.assert_allclose(g[3], e[3], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(g[0], e[0], rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(g[1], e[1], rtol=2e-5, atol=2e-6)
