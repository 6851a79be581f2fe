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
