"""Wire compatibility with reference agents and model files.

Parity is pinned only where the reference ships bytes: the TorchScript archive member
paths of examples/.../cartpole/zmq/client_model.pt (zip listing only -- nothing in it is
unpickled or loaded).  The reference's serde_pickle trajectory frames and libzmq's ZMTP
greeting have no fixture in the reference; the frames below are hand-assembled from the
pickle protocol-3 opcodes serde_pickle emits and from RFC 23 ("parity unpinned" against a
live libzmq / Rust agent, neither of which exists in this image).
"""
import os
import pickle
import socket
import struct
import threading
import time
import zipfile

import numpy as np
import pytest

from relayrl_prototype_amd import _native
from relayrl_prototype_amd.transport import serde_pickle as sp
from relayrl_prototype_amd.types import RelayRLAction, tensordata_json

REF_MODEL = "/root/reference/examples/REINFORCE_without_baseline/classic_control/cartpole/zmq/client_model.pt"


# ---------------------------------------------------------------------- serde_pickle frames
def _opcodes_frame():
    """One CartPole action + the terminal marker, written opcode by opcode the way
    serde_pickle::to_writer lays out Vec<RelayRLAction> (protocol 3, dict per struct,
    Vec<u8> as a list of ints, None for Option::None, unit enum variant as its name)."""
    obs = np.array([0.1, -0.2, 0.03, 0.5], np.float32)
    st = list(tensordata_json(obs)["data"])  # TensorData.data = one-tensor safetensors file

    def s(x):
        b = x.encode()
        return b"X" + struct.pack("<I", len(b)) + b

    def u8list(xs):
        out = b"](" + b"".join(b"K" + bytes([v]) for v in xs) + b"e"
        return out

    act0 = (b"}(" + s("obs") + b"}(" + s("shape") + b"](K\x04e" + s("dtype") + s("Float") + s("data") + u8list(st)
            + b"u" + s("act") + b"N" + s("mask") + b"N" + s("rew") + b"G" + struct.pack(">d", 1.0)
            + s("data") + b"}(" + s("logp_a") + b"}(" + s("Float") + b"G" + struct.pack(">d", -0.69) + b"uu"
            + s("done") + b"\x89" + s("reward_updated") + b"\x88" + b"u")
    last = (b"}(" + s("obs") + b"N" + s("act") + b"N" + s("mask") + b"N" + s("rew") + b"G" + struct.pack(">d", 2.0)
            + s("data") + b"N" + s("done") + b"\x88" + s("reward_updated") + b"\x89" + b"u")
    return b"\x80\x03](" + act0 + last + b"e.", obs


def test_hand_built_serde_pickle_frame_decodes():
    frame, obs = _opcodes_frame()
    assert sp.is_pickle_frame(frame)
    # cross-check the data-only interpreter against CPython on this (trusted, self-made) frame
    assert sp.loads(frame) == pickle.loads(frame)
    acts = sp.actions_from_reference(sp.loads(frame))
    assert len(acts) == 2
    np.testing.assert_array_equal(acts[0].get_obs(), obs)
    assert acts[0].get_rew() == 1.0 and not acts[0].get_done() and acts[0].get_reward_updated()
    assert acts[0].get_data()["logp_a"] == pytest.approx(-0.69)
    assert acts[1].get_obs() is None and acts[1].get_done() and acts[1].get_rew() == 2.0


@pytest.mark.parametrize("dtype_repr", ["Float", ("Float",), {"Float": None}])
def test_enum_representations(dtype_repr):
    obs = np.arange(3, dtype=np.float32)
    td = dict(tensordata_json(obs), dtype=dtype_repr)
    td["data"] = list(td["data"])
    frame = sp.dumps([{"obs": td, "act": None, "mask": None, "rew": 0.5, "data": {"v": ("Double", 1.5)},
                       "done": True, "reward_updated": False}])
    (a,) = sp.actions_from_reference(sp.loads(frame))
    np.testing.assert_array_equal(a.get_obs(), obs)
    assert a.get_data()["v"] == 1.5


def test_reference_frame_roundtrip_matches_cpython():
    acts = [RelayRLAction(np.random.rand(8).astype(np.float32), np.array([2], np.int64), np.ones(4, np.float32),
                          float(i), {"logp_a": np.float32(-1.0), "tag": "x"}, i == 2) for i in range(3)]
    frame = sp.reference_frame(acts)
    assert sp.loads(frame) == pickle.loads(frame)
    back = sp.actions_from_reference(sp.loads(frame))
    for a, b in zip(acts, back):
        np.testing.assert_array_equal(a.get_obs(), b.get_obs())
        np.testing.assert_array_equal(a.get_act(), b.get_act())
        assert a.get_rew() == b.get_rew() and a.get_done() == b.get_done()


@pytest.mark.parametrize("evil", [
    b"\x80\x03cos\nsystem\nX\x02\x00\x00\x00lsR.",          # GLOBAL + REDUCE
    b"\x80\x04\x95\x00\x00\x00\x00\x00\x00\x00\x00\x8c\x02os\x8c\x06system\x93.",  # STACK_GLOBAL
    b"\x80\x02}(X\x01\x00\x00\x00ab.",                      # BUILD
    b"\x80\x03](K\x01",                                     # truncated
])
def test_restricted_interpreter_rejects_code_and_garbage(evil):
    with pytest.raises(sp.PickleFrameError):
        sp.loads(evil)


def test_cumulative_uploads_are_deduplicated():
    mk = lambda i, d=False: RelayRLAction(np.full(4, i, np.float32), np.array([i % 2]), None, 1.0, None, d)  # noqa
    ep1 = [mk(0), mk(1), mk(2, True)]
    ep2 = [mk(10), mk(11, True)]
    dd = sp.CumulativeDeduper()
    assert len(dd.new_actions(ep1)) == 3
    new = dd.new_actions(ep1 + ep2)  # the reference agent re-sends episode 1
    assert [float(a.get_obs()[0]) for a in new] == [10.0, 11.0]
    assert dd.stripped == 3


def test_deduper_keeps_identical_independent_episodes():
    """a deterministic policy from a fixed start state uploads the same episode
    twice -- both are data, not a re-send (the reference never re-sends an upload unchanged)."""
    mk = lambda i, d=False: RelayRLAction(np.full(4, i, np.float32), np.array([i % 2]), None, 1.0, None, d)  # noqa
    ep = [mk(0), mk(1), mk(2, True)]
    dd = sp.CumulativeDeduper()
    assert len(dd.new_actions(ep)) == 3
    assert len(dd.new_actions(list(ep))) == 3
    # a longer upload that merely starts like a remembered one, without an episode boundary there
    part = [mk(0), mk(1)]
    dd2 = sp.CumulativeDeduper()
    dd2.new_actions(part)
    assert len(dd2.new_actions(part + [mk(2, True)])) == 3


def test_pickle_mark_heavy_frame_is_linear():
    """MARK / POP_MARK pairs over a deep stack cost O(1) each (running counter)."""
    body = b"K\x01" * 50000 + b"(1" * 50000
    t0 = time.time()
    with pytest.raises(sp.PickleFrameError):
        sp.loads(b"\x80\x03" + body + b".")  # 50000 values left on the stack at STOP
    assert time.time() - t0 < 2.0


# ---------------------------------------------------------------------- ZMQ endpoint
class _Store:
    def __init__(self):
        self.subs = []
        self.blob = None

    def subscribe(self, fn):
        self.subs.append(fn)

    def unsubscribe(self, fn):
        self.subs.remove(fn)

    def latest(self):
        return self.blob


class _Service:
    def __init__(self):
        self.store = _Store()
        self.got = []
        self.agents = []

    def submit(self, traj, **kw):
        self.got.append(traj)
        return True

    def register_agent(self, a, info=None):
        self.agents.append(a)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _blob():
    import torch

    from relayrl_prototype_amd.ops import MLPSpec
    from relayrl_prototype_amd.runtime.model_store import ModelBlob

    pi = MLPSpec(4, 128, 2).init(torch.Generator().manual_seed(0)).numpy()
    return ModelBlob(3, {"obs_dim": 4, "act_dim": 2, "hidden": 128, "discrete": True}, pi)


def test_endpoint_trains_on_reference_frames_and_pushes_models():
    from relayrl_prototype_amd.transport.zmq_transport import ZmqTrainingEndpoint

    svc = _Service()
    svc.store.blob = _blob()
    al, tr, ts = _port(), _port(), _port()
    ep = ZmqTrainingEndpoint(svc, f"tcp://127.0.0.1:{al}", f"tcp://127.0.0.1:{tr}",
                             model_push_addr=f"tcp://127.0.0.1:{ts}")
    agent_pull = _native.ZmtpSocket(_native.SockType.PULL)  # the reference agent BINDS its model PULL
    agent_pull.bind(f"tcp://127.0.0.1:{ts}")
    dealer = _native.ZmtpSocket(_native.SockType.DEALER, b"AGENT_ID-ref")
    push = _native.ZmtpSocket(_native.SockType.PUSH)
    try:
        dealer.connect(f"tcp://127.0.0.1:{al}")
        assert dealer.send([b"", b"GET_MODEL"], 5000)  # reference handshake: no format frame
        rep = dealer.recv(5000)
        assert rep is not None and rep[1][-1][:2] == b"PK"  # TorchScript zip archive
        assert dealer.send([b"", b"MODEL_SET"], 5000)
        assert dealer.recv(5000)[1][-1] == b"ID_LOGGED"
        # cumulative uploads, each from the same agent
        mk = lambda i, d=False: RelayRLAction(np.full(4, i, np.float32), np.array([i % 2]), None, 1.0, None, d)  # noqa
        ep1 = [mk(0), mk(1, True)]
        push.connect(f"tcp://127.0.0.1:{tr}")
        assert push.send([sp.reference_frame(ep1)], 5000)
        assert push.send([sp.reference_frame(ep1 + [mk(5), mk(6, True)])], 5000)
        t0 = time.time()
        while len(svc.got) < 2 and time.time() - t0 < 10:
            time.sleep(0.02)
        assert [len(t.actions) for t in svc.got] == [2, 2]
        assert ep.reference_frames == 2 and ep.bad_frames == 0
        # model update -> PUSH-connected to the agent's bound PULL, one TorchScript frame
        ep._on_model(svc.store.blob)
        msg = agent_pull.recv(10000)
        assert msg is not None and len(msg[1]) == 1
        assert msg[1][0] == svc.store.blob.torchscript()
    finally:
        for s in (dealer, push, agent_pull):
            s.close()
        ep.close()


def test_reference_agents_survive_the_eviction_sweep():
    """a reference agent never heartbeats; after the sweeper's timeout it
    must still receive model pushes (it is registered exempt and refreshed by its uploads)."""
    from relayrl_prototype_amd.runtime.learner_service import LearnerService
    from relayrl_prototype_amd.transport.zmq_transport import ZmqTrainingEndpoint

    class _Algo:
        def get_weights(self):
            b = _blob()
            return {"obs_dim": 4, "act_dim": 2, "hidden": 128, "discrete": True, "version": b.version,
                    "pi": __import__("torch").from_numpy(b.pi), "vf": None}

        def model_bytes(self):
            return _blob().torchscript()

        def receive_trajectory(self, traj):
            return False

    svc = LearnerService(_Algo())
    al, tr, ts = _port(), _port(), _port()
    ep = ZmqTrainingEndpoint(svc, f"tcp://127.0.0.1:{al}", f"tcp://127.0.0.1:{tr}",
                             model_push_addr=f"tcp://127.0.0.1:{ts}")
    agent_pull = _native.ZmtpSocket(_native.SockType.PULL)
    agent_pull.bind(f"tcp://127.0.0.1:{ts}")
    dealer = _native.ZmtpSocket(_native.SockType.DEALER, b"AGENT_ID-ref2")
    try:
        dealer.connect(f"tcp://127.0.0.1:{al}")
        assert dealer.send([b"", b"GET_MODEL"], 5000)
        assert dealer.recv(5000) is not None
        assert dealer.send([b"", b"MODEL_SET"], 5000)
        assert dealer.recv(5000)[1][-1] == b"ID_LOGGED"
        # the agent stays silent far past the timeout: the sweep evicts nothing of it
        svc.agents["AGENT_ID-ref2"]["last_seen"] -= 1000.0
        assert svc.evict_stale(1.0) == []
        assert b"AGENT_ID-ref2" in ep.ref_agents
        ep._on_model(svc.store.latest())
        msg = agent_pull.recv(10000)
        assert msg is not None and msg[1][0][:2] == b"PK"
    finally:
        for s in (dealer, agent_pull):
            s.close()
        ep.close()


# ---------------------------------------------------------------------- ZMTP/3.0 transcripts (RFC 23)
def _greeting(minor=0, libzmq_padding=False):
    g = bytearray(64)
    g[0] = 0xFF
    if libzmq_padding:
        g[8] = 0x01  # libzmq writes a 64-bit length of 1 into the padding (ZMTP 1.0 detection)
    g[9] = 0x7F
    g[10], g[11] = 3, minor
    g[12:16] = b"NULL"
    return bytes(g)


def _ready(sock_type: bytes, identity: bytes = None):
    body = b"\x05READY" + b"\x0bSocket-Type" + struct.pack(">I", len(sock_type)) + sock_type
    if identity is not None:
        body += b"\x08Identity" + struct.pack(">I", len(identity)) + identity
    return b"\x04" + bytes([len(body)]) + body


def _recv_exact(c, n):
    out = b""
    while len(out) < n:
        chunk = c.recv(n - len(out))
        if not chunk:
            raise ConnectionError("closed")
        out += chunk
    return out


def test_zmtp_push_transcript_byte_exact():
    """Our PUSH against a raw-socket peer that plays libzmq 4.3's PULL side."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    push = _native.ZmtpSocket(_native.SockType.PUSH)
    push.connect(f"tcp://127.0.0.1:{port}")
    c, _ = srv.accept()
    c.settimeout(10)
    try:
        assert _recv_exact(c, 64) == _greeting(0)  # ZMTP 3.0, NULL mechanism, as-server 0
        c.sendall(_greeting(1, libzmq_padding=True))
        ready = _ready(b"PUSH")
        assert _recv_exact(c, len(ready)) == ready
        c.sendall(_ready(b"PULL"))
        threading.Thread(target=lambda: push.send([b"hello", b"x" * 300], 5000), daemon=True).start()
        # short frame with MORE, then a long frame (8-byte size) without
        assert _recv_exact(c, 7) == b"\x01\x05hello"
        assert _recv_exact(c, 9 + 300) == b"\x02" + struct.pack(">Q", 300) + b"x" * 300
    finally:
        c.close()
        srv.close()
        push.close()


def test_zmtp_router_accepts_libzmq_dealer_transcript():
    """A raw-socket libzmq-style DEALER (reference agent) does GET_MODEL against our ROUTER."""
    router = _native.ZmtpSocket(_native.SockType.ROUTER)
    port = router.bind("tcp://127.0.0.1:0")
    c = socket.create_connection(("127.0.0.1", port), timeout=10)
    try:
        c.sendall(_greeting(1, libzmq_padding=True))
        assert _recv_exact(c, 64) == _greeting(0)
        c.sendall(_ready(b"DEALER", b"AGENT_ID-42"))
        ready = _ready(b"ROUTER", b"")
        assert _recv_exact(c, len(ready)) == ready
        c.sendall(b"\x01\x00" + b"\x00\x09GET_MODEL")  # ["", "GET_MODEL"]
        msg = router.recv(5000)
        assert msg is not None
        peer, frames = msg
        assert peer == b"AGENT_ID-42" and frames == [b"", b"GET_MODEL"]
        assert router.send([peer, b"", b"model-bytes"], 5000)
        assert _recv_exact(c, 2 + 13) == b"\x01\x00" + b"\x00\x0bmodel-bytes"
    finally:
        c.close()
        router.close()


# ---------------------------------------------------------------------- TorchScript archive
def _members(path_or_bytes):
    import io

    z = zipfile.ZipFile(path_or_bytes if isinstance(path_or_bytes, str) else io.BytesIO(path_or_bytes))
    return z.namelist()


@pytest.mark.skipif(not os.path.exists(REF_MODEL), reason="reference checkout not present")
def test_torchscript_archive_layout_matches_reference(tmp_path):
    import subprocess
    import sys

    # fresh interpreter: TorchScript's ___torch_mangle_N numbering depends on process history
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from relayrl_prototype_amd.models.policies import PolicyWithoutBaseline, export_torchscript\n"
            "export_torchscript(PolicyWithoutBaseline(4, 2), %r)\n") % (
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), str(tmp_path / "server_model.pt"))
    subprocess.run([sys.executable, "-c", code], check=True)
    ours = _members(str(tmp_path / "server_model.pt"))
    ref = _members(REF_MODEL)
    assert "server_model/code/__torch__/REINFORCE/kernel.py" in ours
    assert {m for m in ours if "/code/" in m} == {m for m in ref if "/code/" in m}
    assert {m for m in ours if "/data/" in m} == {m for m in ref if "/data/" in m}  # W1 b1 W2 b2 W3 b3
    import torch

    m = torch.jit.load(str(tmp_path / "server_model.pt"))
    assert m.get_input_dim() == 4 and m.get_output_dim() == 2
