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
