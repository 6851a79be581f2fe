"""End-to-end agent <-> training server over the local, ZMTP and gRPC transports (CPU).

This is the reference's notebook flow (cartpole_zmq.ipynb:37-97) as a test: a server
and an agent in one process, episodes of a CartPole env, the learner updating every
``traj_per_epoch`` episodes and the agent receiving the new model.
"""
import json
import os
import socket

import numpy as np
import pytest

from relayrl_prototype_amd import _native
from relayrl_prototype_amd.api.agent import RelayRLAgent
from relayrl_prototype_amd.api.server import TrainingServer
from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT


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
    cfg["algorithms"]["REINFORCE"]["traj_per_epoch"] = 4
    cfg["algorithms"]["REINFORCE"]["train_vf_iters"] = 3
    cfg["server"]["training_server"]["port"] = str(free_port())
    cfg["server"]["trajectory_server"]["port"] = str(free_port())
    cfg["server"]["agent_listener"]["port"] = str(free_port())
    p = tmp_path / "relayrl_config.json"
    p.write_text(json.dumps(cfg))
    return tmp_path, str(p)


def run_episodes(agent, n, max_steps=200):
    env = _native.VecEnv("CartPole-v1", 1, 3, 1)
    obs = np.zeros((1, 4), np.float32)
    rew = np.zeros(1, np.float32)
    done = np.zeros(1, np.float32)
    act = np.zeros(1, np.int32)
    env.reset_ptr(obs.ctypes.data)
    lens = []
    for _ in range(n):
        r, steps = 0.0, 0
        while True:
            a = agent.request_for_action(obs[0].copy(), np.ones(2, np.float32), r)
            act[0] = int(np.asarray(a.get_act()).reshape(-1)[0])
            env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
            r = float(rew[0])
            steps += 1
            if done[0] > 0 or steps >= max_steps:
                agent.flag_last_action(r, done=bool(done[0] > 0), truncated=not bool(done[0] > 0))
                break
        lens.append(steps)
    return lens


@pytest.mark.parametrize("server_type,wire", [("local", "columns"), ("zmq", "columns"), ("grpc", "columns"),
                                              ("zmq", "actions"), ("grpc", "actions")])
def test_agent_server_roundtrip(cfgdir, server_type, wire):
    tmp, cfgp = cfgdir
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp / "env"), config_path=cfgp,
                         server_type=server_type, device="cpu", hyperparams={"with_vf_baseline": "true"})
    try:
        agent = RelayRLAgent(config_path=cfgp, server_type=server_type, handshake_timeout_s=30, wire_format=wire)
        assert agent.model_version == 0
        run_episodes(agent, 8)
        import time

        t0 = time.time()
        while srv.service.received < 8 and time.time() - t0 < 20:
            time.sleep(0.02)
        assert srv.wait_idle(60)
        assert srv.service.updates == 2 and srv.service.errors == 0, srv.service.last_error
        # the agent picks the update up (push / poll / subscription)
        import time

        t0 = time.time()
        while agent.model_version < 2 and time.time() - t0 < 10:
            if server_type == "grpc":
                agent.transport.poll(1.0)
            time.sleep(0.05)
        assert agent.model_version == 2
        np.testing.assert_allclose(agent.policy.pi[0].T.ravel()[:10],
                                   srv.algorithm.learner.pi.params[:10].numpy(), rtol=1e-6)
        # progress.txt written with the reference columns
        logs = list((tmp / "env" / "logs").rglob("progress.txt"))
        assert logs
        header = logs[0].read_text().splitlines()[0].split("\t")
        for col in ("Epoch", "AverageEpRet", "StdEpRet", "MaxEpRet", "MinEpRet", "EpLen", "LossPi",
                    "DeltaLossPi", "AverageVVals", "LossV", "KL", "Entropy"):
            assert col in header, col
        assert srv.restart_server()  # lifecycle keeps learner state
        assert srv.service.updates == 2
        agent.close()
    finally:
        srv.close(save=False)


def test_two_agents_zmq(cfgdir):
    tmp, cfgp = cfgdir
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="zmq",
                         device="cpu", multiactor=True)
    try:
        a1 = RelayRLAgent(config_path=cfgp, server_type="zmq")
        a2 = RelayRLAgent(config_path=cfgp, server_type="zmq")
        run_episodes(a1, 2)
        run_episodes(a2, 2)
        import time

        t0 = time.time()
        while srv.service.received < 4 and time.time() - t0 < 20:
            time.sleep(0.02)
        assert srv.wait_idle(60)
        assert srv.service.updates == 1
        import time

        t0 = time.time()
        while (a1.model_version < 1 or a2.model_version < 1) and time.time() - t0 < 10:
            time.sleep(0.05)
        assert a1.model_version == 1 and a2.model_version == 1  # both got the push (A6 fixed)
        assert len(srv.service.agents) == 2
        a1.close()
        a2.close()
    finally:
        srv.close(save=False)


def test_server_model_file_is_torchscript(cfgdir):
    import torch

    tmp, cfgp = cfgdir
    srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="local",
                         device="cpu")
    try:
        path = srv.cfg.get_server_model_path()
        assert os.path.exists(path)
        m = torch.jit.load(path)
        act, data = m.step(torch.zeros(1, 4), torch.ones(1, 2))
        assert m.get_input_dim() == 4 and m.get_output_dim() == 2 and "logp_a" in data
        # an agent can start from that file
        a = RelayRLAgent(model_path=path, config_path=cfgp, server_type="local")
        assert a.policy.obs_dim == 4
        a.close()
    finally:
        srv.close(save=False)


def test_custom_algorithm_plugin(cfgdir):
    tmp, cfgp = cfgdir
    plug = tmp / "algos" / "MYALGO"
    plug.mkdir(parents=True)
    (plug / "MYALGO.py").write_text(
        "from relayrl_prototype_amd.algorithms.reinforce import REINFORCE\n"
        "class MYALGO(REINFORCE):\n"
        "    CONFIG_NAME = 'REINFORCE'\n"
        "    def exp_name(self):\n"
        "        return 'my-algo'\n")
    srv = TrainingServer("MYALGO", 4, 2, 1000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="local",
                         algorithm_dir=str(tmp / "algos"), device="cpu", hyperparams=["pi_lr=0.01", "bogus 3"])
    try:
        assert type(srv.algorithm).__name__ == "MYALGO"
        assert srv.algorithm.params["pi_lr"] == 0.01
    finally:
        srv.close(save=False)


def test_segment_boundaries_keep_rewards_and_bootstrap_obs(cfgdir):
    """Episodes of exactly max_traj_length and 2 * max_traj_length + 1 steps: every reward
    reaches the learner, only the final segment is done, and cut segments carry s_T."""
    tmp, cfgp = cfgdir
    N = 5
    cfg = json.loads(open(cfgp).read())
    cfg["max_traj_length"] = N
    open(cfgp, "w").write(json.dumps(cfg))
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp / "env"), config_path=cfgp,
                         server_type="local", device="cpu")
    got = []
    srv.service.submit = lambda traj: got.append(traj) or True
    try:
        agent = RelayRLAgent(config_path=cfgp, server_type="local", handshake_timeout_s=30)
        assert agent.max_traj_length == N
        for length in (N, 2 * N + 1):
            got.clear()
            obs_seq = [np.full(4, 0.01 * (k + 1), np.float32) for k in range(length + 1)]
            r = 0.0
            for k in range(length):
                agent.request_for_action(obs_seq[k], None, r)
                r = float(k + 1)  # reward of step k
            agent.flag_last_action(r)
            rews = np.concatenate([np.asarray(c.rew) for c in got])
            np.testing.assert_array_equal(rews, np.arange(1, length + 1, dtype=np.float32))
            dones = np.concatenate([np.asarray(c.done) for c in got])
            assert dones[-1] == 1 and dones[:-1].sum() == 0
            assert [len(c) for c in got] == ([N] if length == N else [N, N, 1])
            for i, c in enumerate(got[:-1]):  # cut segments: s_T = next segment's first observation
                np.testing.assert_array_equal(c.next_obs, got[i + 1].obs[0])
            assert got[-1].next_obs is None
            # the columnar wire form round-trips the bootstrap observation
            from relayrl_prototype_amd.types import TrajectoryColumns

            for c in got:
                d = TrajectoryColumns.decode(c.encode())
                if c.next_obs is None:
                    assert d.next_obs is None
                else:
                    np.testing.assert_array_equal(d.next_obs, c.next_obs)
        agent.close()
    finally:
        srv.close(save=False)


def test_cut_segment_bootstraps_with_shipped_next_obs(cfgdir):
    """The learner's return for a cut segment uses V(next_obs), not V(last acted state)."""
    from relayrl_prototype_amd.algorithms.reinforce import REINFORCE
    from relayrl_prototype_amd.ops import reference as ref
    from relayrl_prototype_amd.types import TrajectoryColumns

    tmp, cfgp = cfgdir
    algo = REINFORCE(env_dir=str(tmp / "env"), config_path=cfgp, obs_dim=4, act_dim=2, buf_size=100,
                     device="cpu", with_vf_baseline=True, train_vf_iters=0, traj_per_epoch=100)
    g = np.random.default_rng(1)
    n = 6
    obs = g.normal(size=(n, 4)).astype(np.float32)
    nxt = g.normal(size=4).astype(np.float32)
    c = TrajectoryColumns(obs, np.zeros((n, 1), np.int32), np.ones(n, np.float32), np.zeros(n, np.uint8),
                          None, np.zeros(n, np.float32), next_obs=nxt)
    algo.receive_trajectory(TrajectoryColumns.decode(c.encode()))
    d = algo.buffer.take("cpu")
    assert d["boot_idx"].tolist() == [n - 1]
    vf = algo.learner.vf.params
    v_next = ref.trunk(vf, torch_tensor(nxt[None]), 4, 128, 1)[0][0, 0].item()
    v_last = ref.trunk(vf, torch_tensor(obs[-1:]), 4, 128, 1)[0][0, 0].item()
    assert abs(v_next - v_last) > 1e-6
    # re-stage and run the learner's scan inputs exactly as train_model does
    algo.receive_trajectory(TrajectoryColumns.decode(c.encode()))
    seen = {}
    import relayrl_prototype_amd.algorithms.trajectory_algo as ta

    orig = ta.scan_flat

    def spy(rew, done, val, boot, gamma, lam):
        seen["boot"] = boot.clone()
        return orig(rew, done, val, boot, gamma, lam)

    ta.scan_flat = spy
    try:
        algo.train_model()
    finally:
        ta.scan_flat = orig
    assert abs(float(seen["boot"][n - 1]) - v_next) < 1e-5


def torch_tensor(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, np.float32))


def test_record_action_steps_the_episode_with_external_actions(cfgdir):
    """RelayRLAgent.record_action (agent_zmq.rs:585-596, ``todo!()`` there): externally chosen
    actions join the episode with their rewards, the policy's log-probability of them and V(obs);
    ``done=True`` uploads the episode like flag_last_action."""
    tmp, cfgp = cfgdir
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp / "env"), config_path=cfgp,
                         server_type="local", device="cpu", hyperparams={"with_vf_baseline": "true"})
    got = []
    srv.service.submit = lambda traj: got.append(traj) or True
    try:
        agent = RelayRLAgent(config_path=cfgp, server_type="local", handshake_timeout_s=30)
        p = agent.policy
        obs = [np.full(4, 0.1 * (k + 1), np.float32) for k in range(4)]
        agent.request_for_action(obs[0], None, 0.0)          # the policy's own step
        a1 = agent.record_action(obs[1], 1, None, 2.0)         # a scripted one
        assert a1.get_act().reshape(-1)[0] == 1 and a1.get_rew() == 2.0
        agent.request_for_action(obs[2], np.array([1, 0], np.float32), 2.0)
        agent.record_action(obs[3], 0, np.array([1, 1], np.float32), 5.0, done=True)
        assert len(got) == 1
        c = got[0]
        np.testing.assert_array_equal(c.obs, np.stack(obs))
        assert list(np.asarray(c.act).reshape(-1)[[1, 3]]) == [1, 0]
        np.testing.assert_array_equal(np.asarray(c.rew)[1:], [2.0, 0.0, 5.0])  # row 2's reward never given
        assert np.asarray(c.done)[-1] == 1
        # the stored log-probability of the scripted action is the policy's
        z = p.logits(obs[1].reshape(1, -1), np.ones((1, 2), np.float32))[0].astype(np.float64)
        lp = z[1] - z.max() - np.log(np.exp(z - z.max()).sum())
        assert abs(float(np.asarray(c.logp)[1]) - lp) < 1e-5
        with pytest.raises(RuntimeError):
            agent.disable_agent()
            agent.record_action(obs[0], 0)
        agent.close()
    finally:
        srv.close(save=False)
