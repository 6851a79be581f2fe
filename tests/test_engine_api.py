"""Device engines behind the reference API: TrainingServer(..., engine=...).

CPU: the host engine (C++ env threads + oracle learner) trained through the API object, with
progress.txt in the reference's columns and every update reaching an attached agent; the
multi-rank path runs its ranks as a torch.distributed.run child over gloo.  The GPU twin
(tests/test_engine_gpu.py) trains CartPole to the 475 threshold through the same call.
"""
import json
import os
import socket

import numpy as np
import pytest

from relayrl_prototype_amd.api.agent import RelayRLAgent
from relayrl_prototype_amd.api.server import TrainingServer
from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT
from relayrl_prototype_amd.runtime.engine import resolve_engine
from relayrl_prototype_amd.utils.logger import read_progress

REF_COLS = ("Epoch", "AverageEpRet", "StdEpRet", "MaxEpRet", "MinEpRet", "EpLen", "LossPi", "DeltaLossPi",
            "AverageVVals", "StdVVals", "MaxVVals", "MinVVals", "LossV", "DeltaLossV", "KL", "Entropy")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def cfgdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    cfg["algorithms"]["REINFORCE"]["with_vf_baseline"] = True
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(free_port())
    p = tmp_path / "relayrl_config.json"
    p.write_text(json.dumps(cfg))
    return tmp_path, str(p)


def test_resolve_engine_precedence():
    ap = {"gamma": 0.98, "lam": 0.97, "pi_lr": 3e-4, "vf_lr": 1e-3, "train_vf_iters": 80, "with_vf_baseline": True,
          "seed": 1, "traj_per_epoch": 8, "discrete": True}
    mi = {"engine": "vec", "envs_per_actor": 2048, "rollout_len": 32, "world_size": 4}
    spec = resolve_engine("REINFORCE", 4, 2, ap, mi, {"vf_lr": 1e-2, "num_envs": 512})
    assert spec.kind == "vec" and spec.env == "CartPole-v1" and spec.world_size == 4 and spec.algo == "reinforce"
    t = spec.trainer
    assert t["gamma"] == 0.98 and t["lam"] == 0.97 and t["train_vf_iters"] == 80 and t["with_baseline"] is True
    assert t["vf_lr"] == 1e-2 and t["num_envs"] == 512 and t["rollout_len"] == 32  # hyperparams beat the config
    assert resolve_engine("REINFORCE", 4, 2, ap, {}, {}) is None  # no engine -> trajectory learner
    assert resolve_engine("PPO", 17, 6, ap, {}, {}, engine="vec").env == "HalfCheetahSynth-v0"
    with pytest.raises(ValueError):
        resolve_engine("REINFORCE", 5, 5, ap, {}, {}, engine="vec")  # no env with those dims
    with pytest.raises(ValueError):
        resolve_engine("REINFORCE", 4, 2, ap, {}, {}, engine="warp")


def test_training_server_host_engine_cpu(cfgdir):
    tmp, cfgp = cfgdir
    hp = {"num_envs": 16, "rollout_len": 16, "train_vf_iters": 2, "num_threads": 1}
    srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="local",
                         device="cpu", hyperparams=hp, engine="host")
    try:
        agent = RelayRLAgent(config_path=cfgp, server_type="local", handshake_timeout_s=30)
        assert agent.model_version == 0
        res = srv.train(epochs=3)
        assert res.epochs == 3 and res.env_steps == 3 * 16 * 16
        assert srv.model_version == 3 and agent.model_version == 3
        # the agent acts with the engine's current policy
        np.testing.assert_allclose(agent.policy.pi[0].T.ravel()[:8],
                                   srv.algorithm.learner.pi.params[:8].numpy(), rtol=1e-6)
        a = agent.request_for_action(np.zeros(4, np.float32), None, 0.0)
        assert int(np.asarray(a.get_act()).reshape(-1)[0]) in (0, 1)
        prog = list((tmp / "env" / "logs").rglob("progress.txt"))
        assert len(prog) == 1
        header = prog[0].read_text().splitlines()[0].split("\t")
        for c in REF_COLS:
            assert c in header, c
        cols = read_progress(str(prog[0]))
        assert cols["Epoch"] == [1.0, 2.0, 3.0] and cols["AgentRows"] == [0.0, 0.0, 0.0]
        # agent uploads are staged and folded into the NEXT engine epoch as extra rows
        for t in range(4):
            agent.request_for_action(np.full(4, 0.01 * t, np.float32), None, 1.0)
        agent.flag_last_action(1.0)
        assert srv.wait_idle(10)
        assert srv.algorithm.agent_trajectories == 1 and srv.algorithm.ignored_trajectories == 0
        srv.train(epochs=1)
        rl = srv.algorithm.trainer.rl
        assert rl.last_agent_rows == 5  # the episode's 5 actions (the first one acted above)
        lr = srv.algorithm.learner
        assert int(lr.vloop.loss_last[:, 5].sum().item()) == 16 * 16 + 5  # the value loss counted them
        cols = read_progress(str(prog[0]))
        assert cols["AgentRows"][-1] == 5.0 and cols["AgentEpRet"][-1] == 5.0
        with pytest.raises(RuntimeError):
            TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp / "env2"), config_path=cfgp,
                           server_type="local", training_port=str(free_port()), device="cpu").train(epochs=1)
        agent.close()
    finally:
        srv.close(save=True)
    assert os.path.exists(srv.cfg.get_server_model_path())  # TorchScript export on close


def test_training_server_engine_from_config_block(cfgdir):
    tmp, cfgp = cfgdir
    cfg = json.loads(open(cfgp).read())
    cfg["mi355x"] = {"engine": "host", "envs_per_actor": 8, "rollout_len": 8, "num_threads": 1}
    cfg["algorithms"]["REINFORCE"]["train_vf_iters"] = 1
    open(cfgp, "w").write(json.dumps(cfg))
    srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="local",
                         device="cpu")
    try:
        assert srv.engine_spec.kind == "host" and srv.engine_spec.trainer["num_envs"] == 8
        res = srv.train(epochs=2, log_every=2, publish_every=2)
        assert res.epochs == 2 and srv.model_version == 2
        # the threshold metric as progress columns: NaN until reached, then the TTT itself
        res = srv.train(epochs=30, target_return=1.0, window=1)
        assert res.solved and res.time_to_threshold_s is not None
        cols = read_progress(str(next((tmp / "env" / "logs").rglob("progress.txt"))))
        ttt = cols["TimeToThreshold"]
        assert ttt[-1] == pytest.approx(res.time_to_threshold_s, rel=1e-3)
        assert all(v != v for v in ttt[:-1]) and cols["WindowRet"][-1] >= 1.0
    finally:
        srv.close(save=False)


def test_training_server_multi_rank_engine_gloo(cfgdir, monkeypatch):
    """world_size 2: the ranks run in a torch.distributed.run child; rank 0's policies reach the
    API process (and its agents) over the in-memory relay, never through files."""
    tmp, cfgp = cfgdir
    monkeypatch.setenv("RRL_DIST_BACKEND", "gloo")
    hp = {"num_envs": 8, "rollout_len": 8, "train_vf_iters": 1, "num_threads": 1, "world_size": 2}
    srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="local",
                         device="cpu", hyperparams=hp, engine="host")
    try:
        agent = RelayRLAgent(config_path=cfgp, server_type="local", handshake_timeout_s=30)
        res = srv.train(epochs=2)
        assert res.epochs == 2 and res.env_steps == 2 * 8 * 8 * 2  # both ranks' envs
        assert srv.model_version == 2 and agent.model_version == 2
        prog = list((tmp / "env" / "logs").rglob("progress.txt"))
        assert len(prog) == 1  # rank 0 logs
        assert read_progress(str(prog[0]))["Epoch"] == [1.0, 2.0]
        # a second run continues the version sequence
        srv.train(epochs=1)
        assert srv.model_version == 3 and agent.model_version == 3
        agent.close()
    finally:
        srv.close(save=False)
    assert not list((tmp / "env").rglob("*.safetensors"))  # no weight files anywhere


def drive_agent_against_background_engine(srv, agent, env_dir, seconds: float = 90.0):
    """Background training + one agent stepping CartPole episodes until rank 0's progress.txt
    shows folded agent rows and the agent has seen >= 2 model updates; then stop the ranks.
    Returns (versions seen, AgentRows column, TrainResult)."""
    import time

    from relayrl_prototype_amd import _native

    srv.train(max_seconds=seconds + 30, background=True)
    env = _native.VecEnv("CartPole-v1", 1, 11, 1)
    obs = np.zeros((1, 4), np.float32)
    rew = np.zeros(1, np.float32)
    done = np.zeros(1, np.float32)
    act = np.zeros(1, np.int32)
    env.reset_ptr(obs.ctypes.data)
    versions = [agent.model_version]
    rows = []
    t0 = time.time()
    while time.time() - t0 < seconds:
        r = 0.0
        while True:
            a = agent.request_for_action(obs[0].copy(), np.ones(2, np.float32), r)
            act[0] = int(np.asarray(a.get_act()).reshape(-1)[0])
            env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
            r = float(rew[0])
            if done[0] > 0:
                agent.flag_last_action(r)
                break
        if agent.model_version != versions[-1]:
            versions.append(agent.model_version)
        prog = list(env_dir.rglob("progress.txt"))
        if prog:
            rows = read_progress(str(prog[0])).get("AgentRows", [])
        if len(versions) >= 3 and any(v > 0 for v in rows):
            break
        time.sleep(0.01)
    srv.engine.stop()
    res = srv.engine.join(60)
    return versions, rows, res


def test_zmq_agent_feeds_and_follows_a_two_rank_engine(cfgdir, monkeypatch):
    """a ZMQ agent attached to a world_size=2 engine server while it trains in
    the background contributes rows to rank 0's batches (AgentRows > 0 in progress.txt),
    receives increasing model versions, and no file is on the weight path."""
    tmp, cfgp = cfgdir
    monkeypatch.setenv("RRL_DIST_BACKEND", "gloo")
    hp = {"num_envs": 8, "rollout_len": 8, "train_vf_iters": 1, "num_threads": 1, "world_size": 2}
    srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="zmq",
                         device="cpu", hyperparams=hp, engine="host")
    agent = None
    try:
        agent = RelayRLAgent(config_path=cfgp, server_type="zmq", handshake_timeout_s=30, seed=3)
        versions, rows, res = drive_agent_against_background_engine(srv, agent, tmp / "env")
        assert res is not None and res.epochs >= 1
        assert any(v > 0 for v in rows), rows
        assert len(versions) >= 3 and versions == sorted(versions), versions
        assert srv.algorithm.relay.forwarded >= 1 and srv.algorithm.ignored_trajectories == 0
    finally:
        if agent is not None:
            agent.close()
        srv.close(save=False)
    assert not list((tmp / "env").rglob("*.safetensors"))  # the weight path never touched a file
