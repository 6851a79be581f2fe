"""Columnar RRLC episode frames: codec round trip, learner ingestion equivalence with the
per-action path, corruption rejection (types.py TrajectoryColumns / EpisodeRecorder)."""
import numpy as np
import pytest
import torch

from relayrl_prototype_amd.types import EpisodeRecorder, RelayRLTrajectory, TrajectoryColumns


def _episode(rng, n, D=4, A=2, discrete=True):
    rec = EpisodeRecorder(1000)
    for i in range(n):
        act = np.array(rng.integers(0, A)) if discrete else rng.standard_normal(A).astype(np.float32)
        rec.record(rng.standard_normal(D).astype(np.float32), np.asarray(act), np.ones(A, np.float32),
                   np.float32(-0.5 - i * 0.01))
        rec.set_last_reward(float(i % 3))
    return rec


@pytest.mark.parametrize("discrete", [True, False])
def test_rrlc_roundtrip(discrete):
    rng = np.random.default_rng(0)
    c = _episode(rng, 37, discrete=discrete).take("agent-x", 9, done=True)
    b = c.encode()
    assert TrajectoryColumns.is_frame(b)
    d = TrajectoryColumns.decode(b)
    assert d.agent_id == "agent-x" and d.seq == 9 and len(d) == 37
    for k in ("obs", "act", "mask", "rew", "logp", "done"):
        np.testing.assert_array_equal(getattr(d, k), getattr(c, k))
    assert d.done[-1] == 1 and d.done[:-1].sum() == 0
    acts = d.get_actions()
    assert len(acts) == 37 and acts[-1].get_done() and acts[3].get_rew() == 0.0
    # a per-action RRLT conversion carries the same content
    t = RelayRLTrajectory.decode(d.to_trajectory().encode())
    np.testing.assert_allclose(np.stack([a.get_obs() for a in t.get_actions()]), c.obs)


def test_rrlc_rejects_truncated_and_bad_magic():
    rng = np.random.default_rng(1)
    b = _episode(rng, 5).take("a", 0, True).encode()
    with pytest.raises(ValueError):
        TrajectoryColumns.decode(b[:-3])
    with pytest.raises(ValueError):
        TrajectoryColumns.decode(b"XXXX" + b[4:])


def test_recorder_shape_change_rejected():
    rec = EpisodeRecorder(10)
    rec.record(np.zeros(4, np.float32), np.array(1), None, None)
    with pytest.raises(ValueError):
        rec.record(np.zeros(5, np.float32), np.array(1), None, None)


@pytest.mark.parametrize("algo", ["REINFORCE", "PPO"])
def test_columns_and_actions_ingest_identically(tmp_path, monkeypatch, algo):
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    from relayrl_prototype_amd.algorithms.registry import make_algorithm

    def mk():
        torch.manual_seed(0)
        return make_algorithm(algo, env_dir=str(tmp_path), config_path=str(tmp_path / "c.json"), obs_dim=4,
                              act_dim=2, buf_size=10000, device="cpu", traj_per_epoch=3, train_vf_iters=2,
                              train_pi_iters=2, hidden=32)

    a1, a2 = mk(), mk()
    assert torch.equal(a1.learner.pi.params, a2.learner.pi.params)
    rng = np.random.default_rng(3)
    for ep, (n, done) in enumerate([(11, True), (7, False), (13, True)]):
        c = _episode(rng, n).take("ag", ep, done)
        a1.receive_trajectory(TrajectoryColumns.decode(c.encode()))
        a2.receive_trajectory(c.to_trajectory())
    assert a1.epoch == a2.epoch == 1
    torch.testing.assert_close(a1.learner.pi.params, a2.learner.pi.params, rtol=0, atol=0)
    assert a1.last_metrics["LossPi"] == a2.last_metrics["LossPi"]
