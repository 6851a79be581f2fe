"""Reference learner semantics of uploaded episodes (CPU).

* The reference's terminal marker ``(None, None, None, rew, done=True)`` closes a path with
  ``finish_path(last_val=rew)`` (REINFORCE.py:70-95 -> replay_buffer.py:48-79): the marker
  reward is the path's bootstrap V(s_T), discounted by gamma in the returns, and it is
  dropped entirely without a value baseline.  ``EpisodeIngest`` + the flat scan must give
  the same advantages / returns as a float64 replica of that code.
* ``RelayRLAgent.clear_episode()`` in the middle of an episode must also forget the V(s)
  values recorded for the dropped steps (they ride next to the log-probs).
"""
import numpy as np
import pytest
import torch
from scipy.signal import lfilter

from relayrl_prototype_amd.algorithms.trajectory_algo import EpisodeIngest, FlatBuffer
from relayrl_prototype_amd.ops import scan_flat
from relayrl_prototype_amd.types import EpisodeRecorder, RelayRLAction, RelayRLTrajectory


def _discount_cumsum(x, c):
    """BaseReplayBuffer.py:12-27 (scipy lfilter over the reversed sequence), float64."""
    return lfilter([1], [1, float(-c)], np.asarray(x, np.float64)[::-1], axis=0)[::-1]


def _reference_learner(paths, vals, gamma, lam, baseline):
    """float64 replica of REINFORCE.receive_trajectory's store / finish_path loop."""
    adv, ret = [], []
    for (rews, last_val), v in zip(paths, vals):
        if baseline:
            r = np.append(np.asarray(rews, np.float64), last_val)
            vv = np.append(np.asarray(v, np.float64), last_val)
            deltas = r[:-1] + gamma * vv[1:] - vv[:-1]
            adv.append(_discount_cumsum(deltas, gamma * lam))
            ret.append(_discount_cumsum(r, gamma)[:-1])
        else:
            adv.append(_discount_cumsum(rews, gamma * lam))
            ret.append(_discount_cumsum(rews, gamma))
    return np.concatenate(adv), np.concatenate(ret)


def _episode(rng, n, last_val):
    acts = []
    rews = rng.normal(size=n).astype(np.float32)
    for i in range(n):
        acts.append(RelayRLAction(rng.normal(size=4).astype(np.float32), np.array([i % 2], np.int32),
                                  np.ones(2, np.float32), float(rews[i]),
                                  {"logp_a": np.array([-0.7], np.float32)}, False, True))
    acts.append(RelayRLAction(None, None, None, float(last_val), None, True, False))
    t = RelayRLTrajectory(1000, None)
    t.actions = acts
    return t, rews


@pytest.mark.parametrize("baseline", [True, False])
def test_marker_reward_is_the_finish_path_bootstrap(baseline):
    rng = np.random.default_rng(3)
    gamma, lam = 0.98, 0.97
    buf = FlatBuffer(4, 2, 1000, True)
    ing = EpisodeIngest(buf)
    paths, vals = [], []
    for n, last in ((7, 0.0), (5, 2.5), (9, -1.25)):  # terminal (0) and two cut paths (V(s_T))
        traj, rews = _episode(rng, n, last)
        ing.add(traj)
        paths.append((rews, last))
        vals.append(rng.normal(size=n))
    finished = ing.pop_finished()
    assert [round(r, 5) for r, _ in finished] == [round(float(p[0].sum()) + p[1], 5) for p in paths]  # REINFORCE.py:75
    d = buf.take("cpu")
    val = torch.from_numpy(np.concatenate(vals).astype(np.float32)) if baseline else None
    boot = d["boot"]
    if baseline:
        boot = torch.where(torch.isnan(boot), val, boot)
    else:
        boot = torch.zeros_like(boot)  # trajectory_algo.train_model without a value net
    adv, ret, _ = scan_flat(d["rew"], d["done"], val, boot, gamma, lam)
    adv_ref, ret_ref = _reference_learner(paths, vals, gamma, lam, baseline)
    np.testing.assert_allclose(adv.double().numpy(), adv_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret.double().numpy(), ret_ref, rtol=1e-5, atol=1e-5)
    # the marker reward never becomes a step reward
    np.testing.assert_array_equal(d["rew"].numpy(), np.concatenate([p[0] for p in paths]))


def test_episode_recorder_keeps_values_with_rows():
    rec = EpisodeRecorder(16)
    for i in range(3):
        rec.record(np.full(4, i, np.float32), np.array([0], np.int32), None, -0.5, 10.0 + i)
    rec.n = 0  # RelayRLAgent.clear_episode
    rec.record(np.zeros(4, np.float32), np.array([1], np.int32), None, -0.1, 42.0)
    rec.record(np.zeros(4, np.float32), np.array([1], np.int32), None, -0.1, None)
    assert rec.val[0] == 42.0 and np.isnan(rec.val[1])


def test_clear_episode_mid_episode_reference_wire(tmp_path, monkeypatch):
    """After clear_episode() the next reference upload pairs every row with ITS OWN V(s)."""
    import time

    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.transport import serde_pickle as sp
    from tests.test_reference_agent import ScriptedReferenceServer, _config, _our_archive

    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    cfg, path = _config(tmp_path)
    blob, _ = _our_archive(5, with_vf=True)
    srv = ScriptedReferenceServer(cfg, blob)
    agent = None
    try:
        agent = RelayRLAgent(config_path=path, server_type="zmq", wire_format="reference", seed=0)
        assert agent.policy.vf is not None
        for i in range(3):
            agent.request_for_action(np.full(4, 0.3 * (i + 1), np.float32), np.ones(2, np.float32), 1.0)
        agent.clear_episode()
        kept = [np.array([0.05, -0.1, 0.2, -0.3], np.float32) * (i + 1) for i in range(2)]
        for o in kept:
            agent.request_for_action(o, np.ones(2, np.float32), 1.0)
        agent.flag_last_action(1.0)
        t0 = time.time()
        while not srv.frames and time.time() - t0 < 10:
            time.sleep(0.02)
        raw = sp.loads(srv.frames[0])
        acts = sp.actions_from_reference(raw)
        assert len(acts) == 3 and acts[2].get_obs() is None
        for o, a in zip(kept, acts[:2]):
            np.testing.assert_allclose(a.get_obs().reshape(-1), o)
            v_sent = float(np.asarray(a.get_data()["v"]).reshape(-1)[0])
            v_true = float(np.asarray(agent.policy.value(o.reshape(1, -1))).reshape(-1)[0])
            assert v_sent == pytest.approx(v_true, rel=1e-6, abs=1e-6)
    finally:
        if agent is not None:
            agent.close()
        srv.close()
