"""Codec / type round-trips and byte compatibility with the reference formats."""
import json

import numpy as np
import pytest

from relayrl_prototype_amd import _native
from relayrl_prototype_amd.types import RelayRLAction, RelayRLTrajectory


def test_safetensors_byte_identical_to_python_package():
    stn = pytest.importorskip("safetensors.numpy")
    for arr in [np.arange(4, dtype=np.float64), np.ones((2, 3), np.float32), np.array([1, 2], np.int64),
                np.zeros((0,), np.float32), np.arange(7, dtype=np.int16), np.arange(3, dtype=np.uint8),
                np.array([[1, 2], [3, 4]], np.int32)]:
        dt = {np.float64: "Double", np.float32: "Float", np.int64: "Long", np.int16: "Short", np.uint8: "Byte",
              np.int32: "Int"}[arr.dtype.type]
        mine = _native.st_encode(dt, list(arr.shape), arr.tobytes())
        assert mine == stn.save({"tensor": arr})
        back = _native.st_decode(stn.save({"tensor": arr}))
        assert back[0] == dt and back[1] == list(arr.shape) and back[2] == arr.tobytes()


def test_cartpole_obs_tensor_is_104_bytes():
    # CartPole obs f64[4] -> 104 B safetensors file
    assert len(_native.st_encode("Double", [4], np.zeros(4).tobytes())) == 104


def test_safetensors_rejects_garbage():
    with pytest.raises(Exception):
        _native.st_decode(b"\x05\x00")
    with pytest.raises(Exception):
        _native.st_decode(b"\xff" * 8 + b"{}")


def test_action_json_roundtrip_reference_shape():
    a = RelayRLAction(obs=np.array([0.1, -0.2, 0.3, 0.4]), act=np.array([1.0], np.float32),
                      mask=np.ones(2, np.float32), rew=1.5,
                      data={"logp_a": np.array([-0.69], np.float32), "v": 0.25, "tag": "x"}, done=False)
    j = json.loads(a.to_json())
    assert set(j) == {"obs", "act", "mask", "rew", "data", "done", "reward_updated"}
    assert j["obs"]["dtype"] == "Double" and j["obs"]["shape"] == [4] and len(j["obs"]["data"]) == 104
    assert "Tensor" in j["data"]["logp_a"] and j["data"]["v"] == {"Double": 0.25}
    b = RelayRLAction.action_from_json(j)
    np.testing.assert_array_equal(b.get_obs(), a.get_obs())
    assert b.get_obs().dtype == np.float64
    np.testing.assert_array_equal(b.get_data()["logp_a"], a.get_data()["logp_a"])
    assert b.get_rew() == 1.5 and b.get_done() is False


def test_nested_arrays_keep_shape():
    # reference flattened via tolist() and failed on nested arrays (A12)
    a = RelayRLAction(obs=np.arange(12, dtype=np.float32).reshape(3, 4))
    t = RelayRLTrajectory(10, None)
    t.add_action(a)
    d = RelayRLTrajectory.decode(t.encode())
    assert d.actions[0].get_obs().shape == (3, 4)


def test_trajectory_binary_and_json_roundtrip():
    t = RelayRLTrajectory(max_length=5, trajectory_server=None, agent_id="a1")
    for i in range(3):
        t.add_action(RelayRLAction(obs=np.full(4, i, np.float32), act=np.array([i % 2], np.int32), rew=float(i),
                                   data={"logp_a": np.float32(-0.5), "k": i}))
    t.add_action(RelayRLAction(rew=7.0, done=True), send_if_done=False)
    # not sent -> kept until max_length (reference behaviour)
    assert len(t) == 4
    buf = t.encode()
    u = RelayRLTrajectory.decode(buf)
    assert u.agent_id == "a1" and len(u.actions) == 4
    assert u.actions[2].get_data()["k"] == 2 and u.actions[3].get_done()
    j = RelayRLTrajectory.traj_from_json(json.loads(t.to_json()))
    assert len(j.get_actions()) == 4 and j.get_actions()[1].get_rew() == 1.0


def test_trajectory_send_clears(monkeypatch):
    sent = []
    t = RelayRLTrajectory(100, None, sender=sent.append, send_if_done=True)
    t.add_action(RelayRLAction(obs=np.zeros(2), rew=1))
    assert t.add_action(RelayRLAction(rew=2, done=True))
    assert len(sent) == 1 and len(t) == 0
    assert len(RelayRLTrajectory.decode(sent[0]).actions) == 2


def test_rrlt_rejects_truncation():
    t = RelayRLTrajectory(10, None)
    t.add_action(RelayRLAction(obs=np.zeros(3)))
    b = t.encode()
    for cut in (3, len(b) // 2, len(b) - 1):
        with pytest.raises(Exception):
            _native.traj_decode(b[:cut])


def _rrlt_header(n_actions):
    import struct

    return struct.pack("<II", 0x544C5252, 1) + struct.pack("<I", 0) + struct.pack("<I", 1000) + \
        struct.pack("<I", 1) + b"a" + struct.pack("<Q", 0) + struct.pack("<I", n_actions)


def test_rrlt_hostile_counts_and_shapes_are_refused_cheaply():
    """Network-facing RRLT decoder (codec.cpp traj_decode; the fuzz harness found these): a tiny
    frame claiming 2^28 actions is refused before anything is allocated for them (it used to
    reserve ~100 GB), and tensor shapes whose element count overflows, or is negative, or whose
    byte length field wraps, are refused instead of overflowing."""
    import struct
    import time

    t0 = time.perf_counter()
    with pytest.raises(Exception, match="action count"):
        _native.traj_decode(_rrlt_header(1 << 28) + b"\0" * 16)
    assert time.perf_counter() - t0 < 0.5

    def one_tensor_frame(shape, nbytes_field, payload):
        act = struct.pack("<Bf", 1, 0.0)  # has_obs, reward
        act += struct.pack("<BB", 4, len(shape)) + b"".join(struct.pack("<q", d) for d in shape)
        act += struct.pack("<Q", nbytes_field) + payload
        return _rrlt_header(1) + act

    good = one_tensor_frame([2, 2], 16, b"\0" * 16)
    t = _native.traj_decode(good)
    assert t["agent_id"] == "a" and t["actions"][0]["obs"] == ("Float", [2, 2], b"\0" * 16)
    for shape, nb, payload in (([1 << 62, 8], 16, b"\0" * 16),           # count overflows int64
                               ([-4, -1], 16, b"\0" * 16),                # negative dims
                               ([2, 2], (1 << 64) - 1, b"\0" * 16),       # length field wraps
                               ([3], 16, b"\0" * 16)):                    # plain mismatch
        with pytest.raises(Exception):
            _native.traj_decode(one_tensor_frame(shape, nb, payload))
