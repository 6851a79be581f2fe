"""TrainingServer(engine="vec") on the GPU: CartPole to the 475 threshold through the reference
API (SURVEY N26 / §7.3, o3_training_server.rs:78-151), progress.txt in the reference columns,
and the policy reaching an attached agent."""
import json
import socket

import numpy as np
import pytest

from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT
from relayrl_prototype_amd.utils.logger import read_progress

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_vec_engine_trains_cartpole_to_threshold(cuda, tmp_path, monkeypatch):
    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.api.server import TrainingServer

    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(free_port())
    cfg["mi355x"] = {"engine": "vec", "envs_per_actor": 1024, "rollout_len": 64, "use_graphs": False}
    p = tmp_path / "relayrl_config.json"
    p.write_text(json.dumps(cfg))
    hp = {"with_vf_baseline": True, "train_vf_iters": 5, "pi_lr": 1e-2, "vf_lr": 1e-2, "gamma": 0.99, "lam": 0.95,
          "seed": 1}
    srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp_path / "env"), config_path=str(p),
                         server_type="local", hyperparams=hp)
    try:
        assert srv.engine_spec.kind == "vec"
        agent = RelayRLAgent(config_path=str(p), server_type="local", handshake_timeout_s=30)
        res = srv.train(target_return=475.0, max_seconds=60.0)
        assert res.solved, res
        assert res.time_to_threshold_s is not None and res.time_to_threshold_s < 60
        assert res.last_window_return >= 475.0
        assert agent.model_version == srv.model_version == res.epochs
        prog = list((tmp_path / "env" / "logs").rglob("progress.txt"))
        assert len(prog) == 1
        header = prog[0].read_text().splitlines()[0].split("\t")
        for c in ("Epoch", "AverageEpRet", "StdEpRet", "MaxEpRet", "MinEpRet", "EpLen", "LossPi", "DeltaLossPi",
                  "AverageVVals", "LossV", "DeltaLossV", "KL", "Entropy"):
            assert c in header, c
        cols = read_progress(str(prog[0]))
        assert len(cols["Epoch"]) == res.epochs
        # the served policy is the engine's (the agent's C++ policy mirrors the device weights)
        np.testing.assert_allclose(agent.policy.pi[0].T.ravel()[:8],
                                   srv.algorithm.learner.pi.params[:8].cpu().numpy(), rtol=1e-6)
        agent.close()
    finally:
        srv.close(save=False)


def test_vec_engine_folds_agent_uploads_into_the_batch(cuda, tmp_path, monkeypatch):
    """an attached agent's episodes enter the engine's next batch as extra
    rows -- the row count, the value-loss count and the progress.txt column include them."""
    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.api.server import TrainingServer

    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(free_port())
    cfg["mi355x"] = {"engine": "vec", "envs_per_actor": 512, "rollout_len": 16}
    p = tmp_path / "relayrl_config.json"
    p.write_text(json.dumps(cfg))
    hp = {"with_vf_baseline": True, "train_vf_iters": 3, "seed": 2}
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp_path / "env"), config_path=str(p),
                         server_type="local", hyperparams=hp)
    try:
        agent = RelayRLAgent(config_path=str(p), server_type="local", handshake_timeout_s=30)
        srv.train(epochs=1)
        env = _native.VecEnv("CartPole-v1", 1, 9, 1)
        obs = np.zeros((1, 4), np.float32)
        rew = np.zeros(1, np.float32)
        done = np.zeros(1, np.float32)
        act = np.zeros(1, np.int32)
        env.reset_ptr(obs.ctypes.data)
        rows = 0
        for _ in range(3):
            r = 0.0
            while True:
                a = agent.request_for_action(obs[0].copy(), np.ones(2, np.float32), r)
                act[0] = int(np.asarray(a.get_act()).reshape(-1)[0])
                env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
                r = float(rew[0])
                rows += 1
                if done[0] > 0:
                    agent.flag_last_action(r)
                    break
        assert srv.wait_idle(10)
        res = srv.train(epochs=1)
        algo = srv.algorithm
        assert algo.trainer.rl.last_agent_rows == rows and algo.agent_rows_total == rows
        ls = algo.learner.vloop.loss_last
        assert int(ls[:, 5].sum().item()) == 512 * 16 + rows
        assert res.metrics["AgentRows"] == rows and res.metrics["AgentEpisodes"] == 3
        prog = list((tmp_path / "env" / "logs").rglob("progress.txt"))
        assert read_progress(str(prog[0]))["AgentRows"] == [0.0, float(rows)]
        agent.close()
    finally:
        srv.close(save=False)


def test_vec_engine_two_ranks_shared_gpu_serves_a_zmq_agent(cuda, tmp_path, monkeypatch):
    """VERDICT r3 item 2 on the GPU: a world_size=2 vec engine (two gloo ranks sharing the one
    GPU, RRL_FORCE_DEVICE) trains in the background while a ZMQ agent's episodes are relayed to
    rank 0 and folded into its device batch, and the models reach the agent from rank 0's
    memory over the relay."""
    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.api.server import TrainingServer
    from tests.test_engine_api import drive_agent_against_background_engine

    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    monkeypatch.setenv("RRL_DIST_BACKEND", "gloo")
    monkeypatch.setenv("RRL_FORCE_DEVICE", "0")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(free_port())
    p = tmp_path / "relayrl_config.json"
    p.write_text(json.dumps(cfg))
    hp = {"num_envs": 1024, "rollout_len": 16, "train_vf_iters": 4, "world_size": 2, "with_vf_baseline": True}
    srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp_path / "env"), config_path=str(p),
                         server_type="zmq", hyperparams=hp, engine="vec")
    agent = None
    try:
        agent = RelayRLAgent(config_path=str(p), server_type="zmq", handshake_timeout_s=30, seed=5)
        versions, rows, res = drive_agent_against_background_engine(srv, agent, tmp_path / "env", seconds=60.0)
        assert res is not None and res.epochs >= 1
        assert any(v > 0 for v in rows), rows
        assert len(versions) >= 3 and versions == sorted(versions), versions
    finally:
        if agent is not None:
            agent.close()
        srv.close(save=False)
    assert not list((tmp_path / "env").rglob("*.safetensors"))


def test_agent_rows_replay_a_captured_graph(cuda, tmp_path):
    """epochs with folded agent rows replay a captured graph (padded batch,
    device-side row count and loss scale, grad_args.h) and train the same weights as the eager
    concatenated batch, within fp32 summation order; AgentRows stays exact."""
    import torch

    from relayrl_prototype_amd.runtime.engine import EngineAlgorithm, EngineSpec
    from relayrl_prototype_amd.types import TrajectoryColumns

    rng = np.random.default_rng(0)

    def episode(n):
        obs = rng.normal(size=(n, 4)).astype(np.float32) * 0.1
        act = rng.integers(0, 2, size=(n, 1)).astype(np.int32)
        rew = np.ones(n, np.float32)
        done = np.zeros(n, np.uint8)
        done[-1] = 1
        logp = np.full(n, -0.69, np.float32)
        return TrajectoryColumns(obs, act, rew, done, None, logp, "agent-0", 0)

    uploads = {1: [episode(37), episode(12)], 2: [], 3: [episode(150)], 4: [episode(5), episode(60), episode(8)]}
    res = {}
    for graphs in (False, True):
        spec = EngineSpec("vec", "CartPole-v1", "reinforce", 1,
                          {"env": "CartPole-v1", "algo": "reinforce", "num_envs": 256, "rollout_len": 16,
                           "train_vf_iters": 5, "use_graphs": graphs, "seed": 3, "with_baseline": True})
        algo = EngineAlgorithm(spec, str(tmp_path / f"g{int(graphs)}"), device=cuda, log=False, agent_buf_size=512)
        rows, replays = [], []
        for ep in range(5):
            for t in uploads.get(ep, []):
                algo.receive_trajectory(t)
            r0 = algo.learner.graph_replays
            algo.train_model()
            rows.append(int(algo.trainer.rl.last_agent_rows))
            replays.append(algo.learner.graph_replays - r0)
        torch.cuda.synchronize()
        res[graphs] = (algo.learner.pi.params.cpu().clone(), algo.learner.vf.params.cpu().clone(), rows, replays,
                       algo.trainer.rl._pad is not None)
    e, g = res[False], res[True]
    assert e[2] == g[2] == [0, 49, 0, 150, 73]
    assert g[3] == [1, 1, 1, 1, 1] and e[3] == [0, 0, 0, 0, 0]  # every graph-run epoch replayed a graph
    assert g[4] and not e[4]
    torch.testing.assert_close(g[0], e[0], rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(g[1], e[1], rtol=2e-5, atol=2e-6)
