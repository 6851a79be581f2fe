"""RelayRLAgent(server_type="grpc", wire_format="reference"): the reference agent's own gRPC
dialect.

A scripted grpcio server plays the reference tonic training server (training_grpc.rs:580-797):
it answers the handshake ``ClientPoll{first_time: 1}`` -- first with "no model yet", then with
the reference's own shipped ``client_model.pt`` -- records every request, accepts
``SendActions`` with code 1 and answers the agent's follow-up ``ClientPoll{first_time: 0}`` with
an updated archive, always with version 0 like the reference (training_grpc.rs:724,746,775).
The message classes are the hand-built descriptors of rf/proto/relayrl_grpc.proto
(transport/grpc_transport.py).  Parity with the Rust server itself stays unpinned: it cannot be
built here.
"""
import json
import os
import socket
import threading
from concurrent import futures

import numpy as np
import pytest

from relayrl_prototype_amd import _native
from relayrl_prototype_amd.api.agent import RelayRLAgent
from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT
from relayrl_prototype_amd.transport.grpc_transport import (SERVICE, PbModel, PbRequest, PbResponse, PbTrajectory)
from tests.test_reference_agent import REF_PT, _logits, _our_archive

grpc = pytest.importorskip("grpc")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class ScriptedReferenceGrpcServer:
    def __init__(self, port: int, first_model: bytes, update_model: bytes):
        self.first_model = first_model
        self.update_model = update_model
        self.requests = []      # ("poll", first_time, version) / ("send", n_actions)
        self.trajectories = []  # received PbTrajectory messages
        self._lock = threading.Lock()
        self._handshakes = 0
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        h = {"SendActions": grpc.unary_unary_rpc_method_handler(
                 self._send, request_deserializer=PbTrajectory.FromString,
                 response_serializer=PbResponse.SerializeToString),
             "ClientPoll": grpc.unary_unary_rpc_method_handler(
                 self._poll, request_deserializer=PbRequest.FromString,
                 response_serializer=PbModel.SerializeToString)}
        self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, h),))
        self.server.add_insecure_port(f"127.0.0.1:{port}")
        self.server.start()

    def _send(self, req, ctx):
        with self._lock:
            self.requests.append(("send", len(req.actions)))
            self.trajectories.append(req)
        return PbResponse(code=1, message="trajectory received")  # training_grpc.rs:636-641

    def _poll(self, req, ctx):
        with self._lock:
            self.requests.append(("poll", req.first_time, req.version))
            if req.first_time != 0:
                self._handshakes += 1
                if self._handshakes == 1:
                    return PbModel(code=0, version=0)  # "no initial model yet": the agent retries
                return PbModel(code=1, model=self.first_model, version=0)
            if len(self.trajectories) == 1:
                return PbModel(code=1, model=self.update_model, version=0)  # model_ready after training
            return PbModel(code=0, version=0)

    def close(self):
        self.server.stop(0.2).wait(5)


@pytest.mark.skipif(not os.path.exists(REF_PT), reason="reference checkout not mounted")
def test_reference_grpc_wire_against_scripted_server(tmp_path, monkeypatch):
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    port = _port()
    cfg["server"]["training_server"]["port"] = str(port)
    path = tmp_path / "relayrl_config.json"
    path.write_text(json.dumps(cfg))
    update, pi_new = _our_archive(9, with_vf=True)
    srv = ScriptedReferenceGrpcServer(port, open(REF_PT, "rb").read(), update)
    agent = None
    try:
        agent = RelayRLAgent(config_path=str(path), server_type="grpc", wire_format="reference", seed=0,
                             handshake_timeout_s=20)
        # handshake: first_time 1, version 0, retried after "no model" (agent_grpc.rs:318-360)
        assert srv.requests[:2] == [("poll", 1, 0), ("poll", 1, 0)]
        p = agent.policy
        assert (p.obs_dim, p.act_dim, p.hidden) == (4, 2, 128) and p.vf is None
        from relayrl_prototype_amd.utils.checkpoint import import_reference_weights

        pi_ref, _ = import_reference_weights(REF_PT, 4, 2)
        x = np.array([0.1, -0.2, 0.3, 0.05], np.float32)
        np.testing.assert_allclose(np.asarray(p.logits(x)).reshape(-1), _logits(pi_ref, x), rtol=1e-5, atol=1e-5)
        v0 = agent.model_version
        obs = np.array([0.01, -0.02, 0.03, 0.04], np.float32)
        for t in range(4):
            agent.request_for_action(obs + t, np.ones(2, np.float32), 0.0 if t == 0 else 1.0)
        agent.flag_last_action(1.0)
        # one SendActions per episode, then the synchronous ClientPoll{first_time 0, version 0}
        assert srv.requests[2:] == [("send", 5), ("poll", 0, 0)]
        msg = srv.trajectories[0]
        for i, m in enumerate(msg.actions[:4]):
            assert m.reward_update_flag is False and m.done is False and m.reward == 1.0
            dt, shape, raw = _native.st_decode(m.obs)  # one-tensor safetensors files (action.rs:342-352)
            assert shape == [4]
            np.testing.assert_allclose(np.frombuffer(raw, np.float32), obs + i)
            for f in (m.action, m.mask):
                dt_f, _, raw_f = _native.st_decode(f)
                assert dt_f == _native.st_decode(m.obs)[0]  # f32 like obs (the agent casts to Float)
            d = json.loads(m.data["logp_a"].decode())  # RelayRLData JSON, externally tagged
            assert list(d) == ["Tensor"] and d["Tensor"]["dtype"] == "Float"
            assert "v" not in m.data  # PolicyWithoutBaseline's step() dict
        last = msg.actions[4]
        assert last.done is True and not last.obs and not last.action and not last.mask and last.reward == 0.0
        # the poll's non-empty model was swapped in (a PolicyWithBaseline archive now)
        assert agent.model_version == v0 + 1 and agent.policy.vf is not None
        np.testing.assert_allclose(np.asarray(agent.policy.logits(x)).reshape(-1), _logits(pi_new, x), rtol=1e-5,
                                   atol=1e-5)
        # the next episode carries data['v'] for the baseline learner; an empty poll answer keeps the model
        agent.request_for_action(obs, np.ones(2, np.float32), 0.0)
        agent.flag_last_action(0.0)
        assert srv.requests[4:] == [("send", 2), ("poll", 0, 0)]
        assert "v" in srv.trajectories[1].actions[0].data
        assert agent.model_version == v0 + 1
    finally:
        if agent is not None:
            agent.close()
        srv.close()


def test_reference_grpc_wire_trains_against_our_server(tmp_path, monkeypatch):
    """Our gRPC endpoint speaks the reference dialect too: uploads train the learner and the
    follow-up polls return the new models."""
    import time

    from relayrl_prototype_amd.api.server import TrainingServer

    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(_port())
    cfg["algorithms"]["REINFORCE"].update(traj_per_epoch=2, train_vf_iters=2, with_vf_baseline=True)
    path = tmp_path / "relayrl_config.json"
    path.write_text(json.dumps(cfg))
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp_path), config_path=str(path),
                         server_type="grpc", device="cpu")
    agent = None
    try:
        agent = RelayRLAgent(config_path=str(path), server_type="grpc", wire_format="reference", seed=1)
        v0 = agent.model_version
        env = _native.VecEnv("CartPole-v1", 1, 5, 1)
        obs = np.zeros((1, 4), np.float32)
        rew = np.zeros(1, np.float32)
        done = np.zeros(1, np.float32)
        act = np.zeros(1, np.int32)
        env.reset_ptr(obs.ctypes.data)
        for _ in range(6):
            r = 0.0
            while True:
                a = agent.request_for_action(obs[0].copy(), np.ones(2, np.float32), r)
                act[0] = int(np.asarray(a.get_act()).reshape(-1)[0])
                env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
                r = float(rew[0])
                if done[0] > 0:
                    agent.flag_last_action(r)
                    break
            time.sleep(0.05)  # our SendActions queues the upload; give the learner a moment
        srv.wait_idle(60)
        assert srv.service.updates >= 2
        assert agent.model_version >= v0 + 1  # TorchScript archives came back through ClientPoll
    finally:
        if agent is not None:
            agent.close()
        srv.close(save=False)
