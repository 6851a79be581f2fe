"""Property-based fuzzing (hypothesis) of the wire codecs and the host policy: random
shapes / dtypes / lengths must round-trip exactly, malformed frames must be rejected
with an exception (never a crash), and byte compatibility with the `safetensors`
package holds for every dtype the reference supports."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from relayrl_prototype_amd import _native
from relayrl_prototype_amd.types import RelayRLAction, RelayRLTrajectory, TrajectoryColumns

DTYPES = {"Byte": np.uint8, "Short": np.int16, "Int": np.int32, "Long": np.int64, "Float": np.float32,
          "Double": np.float64}
FAST = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@FAST
@given(dt=st.sampled_from(sorted(DTYPES)), shape=st.lists(st.integers(0, 5), min_size=0, max_size=4),
       seed=st.integers(0, 2 ** 31 - 1))
def test_safetensors_roundtrip_and_byte_compat(dt, shape, seed):
    stn = pytest.importorskip("safetensors.numpy")
    rng = np.random.default_rng(seed)
    arr = np.ascontiguousarray(np.asarray(rng.standard_normal(shape) * 100).astype(DTYPES[dt]))
    enc = _native.st_encode(dt, list(arr.shape), arr.tobytes())
    assert enc == stn.save({"tensor": arr})
    d, s, raw = _native.st_decode(enc)
    assert d == dt and list(s) == list(arr.shape) and raw == arr.tobytes()


@FAST
@given(data=st.binary(min_size=0, max_size=200))
def test_decoders_reject_garbage_without_crashing(data):
    for fn in (_native.st_decode, RelayRLTrajectory.decode, TrajectoryColumns.decode):
        try:
            fn(data)
        except Exception:
            pass


@FAST
@given(n=st.integers(0, 40), D=st.integers(1, 9), A=st.integers(1, 5), cont=st.booleans(), mask=st.booleans(),
       seed=st.integers(0, 10 ** 6))
def test_rrlc_columns_roundtrip(n, D, A, cont, mask, seed):
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((n, D)).astype(np.float32)
    act = rng.standard_normal((n, A)).astype(np.float32) if cont else rng.integers(0, A, (n, 1)).astype(np.int32)
    c = TrajectoryColumns(obs, act, rng.standard_normal(n).astype(np.float32),
                          (rng.random(n) < 0.1).astype(np.uint8), rng.random((n, A)).astype(np.float32) if mask else None,
                          rng.standard_normal(n).astype(np.float32), agent_id=f"a{seed}", seq=seed)
    b = c.encode()
    d = TrajectoryColumns.decode(b)
    assert d.agent_id == c.agent_id and d.seq == c.seq and len(d) == n
    for k in ("obs", "act", "rew", "done", "logp"):
        np.testing.assert_array_equal(getattr(d, k), getattr(c, k).reshape(getattr(d, k).shape))
    assert (d.mask is None) == (not mask)
    # any truncation is rejected
    if len(b) > 1:
        with pytest.raises(ValueError):
            TrajectoryColumns.decode(b[:-1])


@FAST
@given(n=st.integers(1, 20), seed=st.integers(0, 10 ** 6))
def test_rrlt_roundtrip_with_aux_data(n, seed):
    rng = np.random.default_rng(seed)
    t = RelayRLTrajectory(1000, None, agent_id="x")
    t.seq = seed
    for i in range(n):
        t.add_action(RelayRLAction(obs=rng.standard_normal(3).astype(np.float32), act=np.array([i % 3], np.int64),
                                   mask=np.ones(3, np.float32), rew=float(rng.standard_normal()),
                                   data={"logp_a": np.float32(rng.standard_normal()), "k": "v", "i": 7},
                                   done=(i == n - 1)), send_if_done=False)
    back = RelayRLTrajectory.decode(t.encode())
    assert back.seq == seed and len(back) == n
    for a, b in zip(t.get_actions(), back.get_actions()):
        np.testing.assert_array_equal(a.get_obs(), b.get_obs())
        assert np.float32(a.get_rew()) == np.float32(b.get_rew()) and a.get_done() == b.get_done()  # f32 on the wire
        assert b.get_data()["k"] == "v" and b.get_data()["i"] == 7


@FAST
@given(D=st.integers(1, 12), A=st.integers(1, 6), H=st.sampled_from([16, 64, 128]), N=st.integers(1, 9),
       seed=st.integers(0, 10 ** 6))
def test_native_policy_matches_numpy_for_any_shape(D, A, H, N, seed):
    import torch

    from relayrl_prototype_amd.models.cpu_policy import CPUPolicy
    from relayrl_prototype_amd.ops.mlp import MLPSpec

    g = torch.Generator().manual_seed(seed)
    p = CPUPolicy(D, A, H, True, MLPSpec(D, H, A).init(g).numpy(), MLPSpec(D, H, 1).init(g).numpy(), seed=1)
    x = np.random.default_rng(seed).standard_normal((N, D)).astype(np.float32)
    np.testing.assert_allclose(p._nat.logits(x), p.logits(x), rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(p._nat.value(x), p.value(x), rtol=2e-5, atol=2e-5)
