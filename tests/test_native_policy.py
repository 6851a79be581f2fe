"""Native C++ agent policy (csrc/host/policy.cpp) vs the numpy fp32 reference."""
import numpy as np
import pytest
import torch

from relayrl_prototype_amd.models.cpu_policy import CPUPolicy
from relayrl_prototype_amd.ops.mlp import MLPSpec


def _policy(discrete, D=6, H=64, A=3, vf=True, seed=0):
    g = torch.Generator().manual_seed(seed)
    pi = MLPSpec(D, H, A, not discrete).init(g).numpy()
    v = MLPSpec(D, H, 1).init(g).numpy() if vf else None
    return CPUPolicy(D, A, H, discrete, pi, v, seed=5)


@pytest.mark.parametrize("discrete", [True, False])
def test_native_forward_matches_numpy(discrete):
    p = _policy(discrete)
    x = np.random.default_rng(1).standard_normal((33, 6)).astype(np.float32)
    np.testing.assert_allclose(p._nat.logits(x), p.logits(x), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(p._nat.value(x), p.value(x), rtol=1e-5, atol=1e-5)
    act, data = p.step(x)
    np.testing.assert_allclose(data["v"], p.value(x), rtol=1e-5, atol=1e-5)
    if discrete:
        lg = p.logits(x)
        lp = lg - np.log(np.exp(lg - lg.max(-1, keepdims=True)).sum(-1, keepdims=True)) - lg.max(-1, keepdims=True)
        np.testing.assert_allclose(data["logp_a"], lp[np.arange(33), act], rtol=1e-4, atol=1e-5)
    else:
        mu, ls = p.logits(x), p.pi[6]
        z = (act - mu) / np.exp(ls)
        ref = (-0.5 * z * z - ls - 0.9189385332046727).sum(-1)
        np.testing.assert_allclose(data["logp_a"], ref, rtol=1e-4, atol=1e-4)


def test_native_categorical_frequencies_and_mask():
    p = _policy(True, vf=False)
    x = np.tile(np.random.default_rng(2).standard_normal((1, 6)).astype(np.float32), (20000, 1))
    act, data = p.step(x)
    assert "v" not in data
    lg = p.logits(x[:1])[0]
    probs = np.exp(lg - lg.max()) / np.exp(lg - lg.max()).sum()
    freq = np.bincount(act, minlength=3) / len(act)
    np.testing.assert_allclose(freq, probs, atol=0.015)
    mask = np.tile(np.array([[1, 0, 1]], np.float32), (2000, 1))
    act, _ = p.step(x[:2000], mask)
    assert not (act == 1).any()


def test_native_gaussian_moments():
    p = _policy(False, vf=False)
    x = np.zeros((20000, 6), np.float32)
    act, _ = p.step(x)
    mu = p.logits(x[:1])[0]
    np.testing.assert_allclose(act.mean(0), mu, atol=0.03)
    np.testing.assert_allclose(act.std(0), np.exp(p.pi[6]), rtol=0.03)


def test_native_policy_rejects_bad_sizes():
    from relayrl_prototype_amd import _native

    n = _native.NativePolicy(4, 16, 2, True)
    with pytest.raises(ValueError):
        n.load(np.zeros(10, np.float32))


@pytest.mark.parametrize("H,A", [(100, 3), (128, 20), (192, 2)])
def test_native_forward_blocked_and_tail_widths(H, A):
    """dense(): 64-wide register blocks plus the axpy tail (H = 100, 192), the dot-product head
    (A < 16) and the transposed head (A = 20)."""
    p = _policy(True, D=5, H=H, A=A)
    x = np.random.default_rng(3).standard_normal((17, 5)).astype(np.float32)
    np.testing.assert_allclose(p._nat.logits(x), p.logits(x), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(p._nat.value(x), p.value(x), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("discrete", [True, False])
@pytest.mark.parametrize("vf", [True, False])
def test_step_row_matches_step_and_writes_the_episode_row(discrete, vf):
    """NativePolicy.step_row (request_for_action's native path): the same draws as step() on
    the same RNG stream, and the row written into the EpisodeRecorder's columns."""
    from relayrl_prototype_amd.types import EpisodeRecorder

    a, b = _policy(discrete, vf=vf), _policy(discrete, vf=vf)
    rec = EpisodeRecorder(8)
    sink = rec.sink(6, discrete, 3)
    rng = np.random.default_rng(4)
    for i in range(8):
        x = rng.standard_normal(6).astype(np.float32)
        m = np.array([1, 0, 1], np.float32) if discrete else np.ones(3, np.float32)
        act, data = a.step(x, m)
        a0, logp, v = b._nat.step_row(x, m, sink, i)
        rec.n += 1
        if discrete:
            assert a0.shape == () and a0.dtype == np.int32 and int(a0) == int(act[0]) and int(a0) != 1
        else:
            assert a0.shape == (3,) and np.array_equal(a0, act[0])
        assert logp.shape == () and logp == data["logp_a"][0]
        if vf:
            assert v.shape == () and v == data["v"][0]
        else:
            assert v is None
        np.testing.assert_array_equal(rec.obs[i], x)
        np.testing.assert_array_equal(rec.mask[i], m)
        np.testing.assert_array_equal(rec.act[i], np.asarray(a0).reshape(-1))
        assert rec.logp[i] == logp and rec.rew[i] == 0 and rec.done[i] == 0
        assert (np.isnan(rec.val[i]) if not vf else rec.val[i] == v)
    with pytest.raises(IndexError):
        b._nat.step_row(x, m, sink, 8)
    with pytest.raises(ValueError):
        b._nat.step_row(np.zeros(5, np.float32), m, sink, 0)
    with pytest.raises(ValueError):  # a sink allocated for the other action kind
        b._nat.step_row(x, m, EpisodeRecorder(4).sink(6, not discrete, 3), 0)


def test_agent_fast_path_records_what_it_returns(tmp_path):
    from relayrl_prototype_amd.api.agent import RelayRLAgent

    p = _policy(True)
    ag = RelayRLAgent.__new__(RelayRLAgent)  # the step path only: no transport
    import threading

    from relayrl_prototype_amd.types import EpisodeRecorder

    ag.enabled, ag.policy, ag._policy_lock, ag._rec, ag._aux = True, p, threading.Lock(), EpisodeRecorder(16), []
    rng = np.random.default_rng(6)
    xs = rng.standard_normal((5, 6))  # float64 in, float32 recorded
    for k, x in enumerate(xs):
        act = ag.request_for_action(x, None, float(k))
        assert act.get_obs().dtype == np.float32 and np.array_equal(act.get_obs(), x.astype(np.float32))
        assert set(act.get_data()) == {"logp_a", "v"}
    r = ag._rec
    assert r.n == 5
    np.testing.assert_array_equal(r.obs[:5], xs.astype(np.float32))
    np.testing.assert_array_equal(r.rew[:4], [1, 2, 3, 4])  # each reward lands on the previous action


def test_record_action_gaussian_log_prob():
    """record_action with a Gaussian policy: the stored log-probability is the policy's density of
    the given action, the row's reward the one passed."""
    import threading

    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.types import EpisodeRecorder

    p = _policy(False)
    ag = RelayRLAgent.__new__(RelayRLAgent)
    ag.enabled, ag.policy, ag._policy_lock, ag._rec, ag._aux = True, p, threading.Lock(), EpisodeRecorder(8), []
    x = np.random.default_rng(7).standard_normal(6).astype(np.float32)
    a = np.array([0.3, -0.2, 0.9], np.float32)
    ag.record_action(x, a, None, 1.5)
    mu, ls = p.logits(x.reshape(1, -1))[0].astype(np.float64), p.pi[6].astype(np.float64)
    z = (a - mu) / np.exp(ls)
    want = (-0.5 * z * z - ls - 0.9189385332046727).sum()
    r = ag._rec
    assert r.n == 1 and r.rew[0] == 1.5 and abs(r.logp[0] - want) < 1e-4
    np.testing.assert_array_equal(r.act[0], a)
    assert abs(r.val[0] - p.value(x.reshape(1, -1))[0]) < 1e-5
