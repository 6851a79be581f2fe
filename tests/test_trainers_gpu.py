"""Trainers and algorithms on the MI355X through the HIP kernels."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_vec_trainer_graph_equals_eager(cuda):
    """hipGraph-captured value loop gives bit-identical parameters to eager launches."""
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    res = []
    for graphs in (True, False):
        cfg = VecTrainerConfig(num_envs=512, rollout_len=32, train_vf_iters=5, use_graphs=graphs, seed=4)
        tr = VecTrainer(cfg)
        for _ in range(3):
            tr.train_epoch()
        torch.cuda.synchronize()
        res.append((tr.pi.params.clone(), tr.vf.params.clone(), int(tr.vf.step.item())))
    assert res[0][2] == res[1][2] == 15
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_average_ep_return_matches_metrics(cuda):
    """The one-read threshold check of bench.py's time-to-threshold loop returns exactly
    metrics()["AverageEpRet"] (NaN before the first finished episode)."""
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    tr = VecTrainer(VecTrainerConfig(num_envs=1024, rollout_len=64, train_vf_iters=3, seed=2))
    seen = 0
    for _ in range(4):
        tr.train_epoch()
        fast = tr.average_ep_return()
        full = tr.metrics()["AverageEpRet"]
        if full != full:
            assert fast != fast
        else:
            seen += 1
            assert fast == full
    assert seen > 0


@pytest.mark.parametrize("algo", ["reinforce", "a2c", "ppo"])
def test_vec_trainer_algos(cuda, algo):
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    cfg = VecTrainerConfig(num_envs=1024, rollout_len=32, algo=algo, train_vf_iters=4, train_pi_iters=4,
                           target_kl=0.05 if algo == "ppo" else None, ent_coef=0.01 if algo == "a2c" else 0.0)
    tr = VecTrainer(cfg)
    for _ in range(3):
        tr.train_epoch()
    m = tr.metrics()
    assert math.isfinite(m["LossPi"]) and math.isfinite(m["LossV"]) and m["Episodes"] > 0


def test_vec_trainer_cartpole_solves(cuda):
    """Convergence: CartPole-v1 average return >= 475 (the gymnasium threshold)."""
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    cfg = VecTrainerConfig(num_envs=4096, rollout_len=128, with_baseline=True, pi_lr=1e-2, vf_lr=3e-3,
                           train_vf_iters=20, gamma=0.99, lam=0.95, seed=7)
    tr = VecTrainer(cfg)
    best = 0.0
    for ep in range(150):
        tr.train_epoch()
        m = tr.metrics()
        if m["Episodes"]:
            best = max(best, m["AverageEpRet"])
        if best >= 475:
            break
    assert best >= 475, (best, ep)


@pytest.mark.parametrize("env,algo", [("CartPole-v1", "reinforce"), ("HalfCheetahSynth-v0", "ppo"),
                                      ("LunarLanderSynth-v0", "a2c")])
def test_host_trainer_gpu(cuda, env, algo):
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    cfg = HostTrainerConfig(env=env, num_envs=256, rollout_len=32, algo=algo, train_vf_iters=4, train_pi_iters=4,
                            num_threads=8)
    tr = HostVecTrainer(cfg)
    p0 = tr.learner.pi.params.clone()
    for _ in range(2):
        tr.train_epoch()
    m = tr.metrics()
    assert math.isfinite(m["LossPi"]) and not torch.equal(p0, tr.learner.pi.params)
    # the device-sampled actions were what the envs received
    if env == "CartPole-v1":
        assert torch.equal(tr.h_act.to(cuda), tr.d_act)


def test_trajectory_reinforce_on_gpu(cuda, tmp_path, monkeypatch):
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    from relayrl_prototype_amd.algorithms.registry import make_algorithm
    from relayrl_prototype_amd.types import RelayRLAction, RelayRLTrajectory

    alg = make_algorithm("REINFORCE", env_dir=str(tmp_path), config_path=str(tmp_path / "c.json"), obs_dim=4,
                         act_dim=2, buf_size=10000, device="cuda", traj_per_epoch=2, train_vf_iters=3,
                         with_vf_baseline=True)
    rng = np.random.default_rng(0)
    for ep in range(2):
        t = RelayRLTrajectory(1000, None)
        for s in range(50):
            t.add_action(RelayRLAction(obs=rng.standard_normal(4), act=np.array([rng.integers(0, 2)]),
                                       mask=np.ones(2), rew=1.0, data={"logp_a": np.float32(-0.69)}, done=(s == 49)))
        up = alg.receive_trajectory(t)
    assert up and alg.learner.pi.params.is_cuda
    assert math.isfinite(alg.last_metrics["LossPi"]) and math.isfinite(alg.last_metrics["LossV"])


def test_agent_server_zmq_with_gpu_learner(cuda, tmp_path, monkeypatch):
    """Notebook flow with the learner on the MI355X: columnar uploads over ZMTP feed the
    HIP learner; the new weights reach the agent's C++ policy."""
    import json
    import socket
    import time

    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.api.server import TrainingServer
    from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT

    def port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    cfg["algorithms"]["REINFORCE"]["traj_per_epoch"] = 4
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(port())
    (tmp_path / "c.json").write_text(json.dumps(cfg))
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp_path), config_path=str(tmp_path / "c.json"),
                         server_type="zmq", device="cuda", hyperparams={"with_vf_baseline": "true"})
    try:
        assert srv.algorithm.learner.pi.params.is_cuda
        agent = RelayRLAgent(config_path=str(tmp_path / "c.json"), server_type="zmq")
        env = _native.VecEnv("CartPole-v1", 1, 0, 1)
        obs = np.zeros((1, 4), np.float32)
        rew = np.zeros(1, np.float32)
        done = np.zeros(1, np.float32)
        act = np.zeros(1, np.int32)
        env.reset_ptr(obs.ctypes.data)
        for _ in range(8):
            r = 0.0
            while True:
                a = agent.request_for_action(obs[0], None, r)
                act[0] = int(np.asarray(a.get_act()).reshape(-1)[0])
                env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
                r = float(rew[0])
                if done[0] > 0:
                    agent.flag_last_action(r)
                    break
        t0 = time.time()
        while srv.service.received < 8 and time.time() - t0 < 30:
            time.sleep(0.02)
        assert srv.wait_idle(60) and srv.service.updates == 2, srv.service.last_error
        t0 = time.time()
        while agent.model_version < 2 and time.time() - t0 < 10:
            time.sleep(0.05)
        assert agent.model_version == 2
        np.testing.assert_allclose(agent.policy.pi[0].T.ravel()[:10],
                                   srv.algorithm.learner.pi.params[:10].cpu().numpy(), rtol=1e-6)
        agent.close()
    finally:
        srv.close(save=False)


def hip_cus_limit() -> int:
    from relayrl_prototype_amd.ops import hip

    h = hip()
    prev = h.set_cu_limit(0)
    h.set_cu_limit(prev)
    return prev


def test_host_trainer_overlap_lag1(cuda):
    """Lag-1 host pipeline: rollout k+1 acts with the policy of update k-1 while update k runs,
    every epoch learns exactly one rollout, and the buffers alternate."""
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    cfg = HostTrainerConfig(env="CartPole-v1", num_envs=512, rollout_len=32, train_vf_iters=4, num_threads=4,
                            overlap=True, seed=2, actor_cus=16)
    tr = HostVecTrainer(cfg, device=cuda)
    assert tr.overlap and len(tr.bufs) == 2
    for _ in range(4):
        tr.train_epoch()
    tr.finish()
    torch.cuda.synchronize()
    assert tr.snapshot_versions == [0, 0, 1, 2, 3]  # REINFORCE: one policy step per epoch
    m = tr.metrics()
    assert m["EnvSteps"] == 4 * 512 * 32
    assert math.isfinite(m["LossPi"]) and torch.isfinite(tr.learner.pi.params).all()
    assert tr.cu_split[0] == 16 and hip_cus_limit() == tr.cu_split[1]
    tr.close()
    assert hip_cus_limit() == 0


def test_host_trainer_overlap_learns(cuda):
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    cfg = HostTrainerConfig(env="CartPole-v1", num_envs=256, rollout_len=100, algo="ppo", pi_lr=3e-3, vf_lr=3e-3,
                            train_vf_iters=10, train_pi_iters=10, num_threads=4, seed=0, overlap=True)
    tr = HostVecTrainer(cfg, device=cuda)
    best = 0.0
    for _ in range(40):
        tr.train_epoch()
        m = tr.metrics()
        if m["Episodes"]:
            best = max(best, m["AverageEpRet"])
        if best > 150:
            break
    tr.close()
    assert best > 150, best


@pytest.mark.parametrize("overlap", [False, True])
def test_host_trainer_no_sync_equals_synced(cuda, overlap):
    """without a host sync between epochs (log_every > 1) the next rollout's first
    H2D copy must still wait for the previous update's reads of that buffer set.  The run
    with a synchronize() after every epoch is the race-free reference; both must agree
    bit for bit (every kernel here is deterministic)."""
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    def run(sync_every_epoch):
        cfg = HostTrainerConfig(env="CartPole-v1", num_envs=2048, rollout_len=16, train_vf_iters=20, num_threads=4,
                                overlap=overlap, seed=5)
        tr = HostVecTrainer(cfg, device=cuda)
        for _ in range(6):
            tr.train_epoch()
            if sync_every_epoch:
                torch.cuda.synchronize()
        tr.close()
        torch.cuda.synchronize()
        return tr.learner.pi.params.clone(), tr.learner.vf.params.clone()

    p_sync, v_sync = run(True)
    p_fast, v_fast = run(False)
    assert torch.equal(p_sync, p_fast) and torch.equal(v_sync, v_fast)


@pytest.mark.parametrize("env", ["CartPole-v1", "HalfCheetahSynth-v0"])
def test_native_host_rollout_matches_python_loop(cuda, env):
    """The C++ rollout driver (csrc/runtime/host_rollout.cpp: zero-copy sampling launches,
    env threads stepped from C++) produces bit for bit the rollout of the Python loop
    (same Philox streams, same env seeds), and the learner then agrees exactly."""
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    def run(native):
        cfg = HostTrainerConfig(env=env, num_envs=1000, rollout_len=24, train_vf_iters=3, num_threads=4, seed=3,
                                algo="ppo" if env.startswith("Half") else "reinforce", train_pi_iters=2,
                                native_rollout=native)
        tr = HostVecTrainer(cfg, device=cuda)
        assert (tr.driver is not None) == native
        outs = []
        for _ in range(3):
            tr.train_epoch()
            torch.cuda.synchronize()
            outs.append([x.clone() for x in (tr.d_obs, tr.d_act, tr.d_logp, tr.d_rew, tr.d_done)])
        m = tr.metrics()
        return outs, tr.learner.pi.params.clone(), m

    o_nat, p_nat, m_nat = run(True)
    o_py, p_py, _ = run(False)
    for a, b in zip(o_nat, o_py):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    assert torch.equal(p_nat, p_py)
    assert m_nat["HostStepUs"] > 0 and m_nat["HostEnvWaitUs"] >= 0


def test_halfcheetah_ppo_chunked_big_batch(cuda):
    """A 39 M-transition PPO epoch (HalfCheetahSynth, 65,536 envs x 600 steps): the fused
    fwd+bwd launches split at GRAD_CHUNK_ROWS (2 chunks), 64-bit buffer addressing in the
    rollout / forward / scan kernels (obs buffer 2.7 GB, > 2^31 floats' byte offsets), and the
    GAE scan of sampled columns against the float64 oracle."""
    from relayrl_prototype_amd.ops import mlp as mlpops
    from relayrl_prototype_amd.ops import reference as ref
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    T, N = 600, 65536
    assert len(mlpops.grad_chunks(T * N)) == 2
    cfg = VecTrainerConfig(env="HalfCheetahSynth-v0", algo="ppo", num_envs=N, rollout_len=T, train_pi_iters=2,
                           train_vf_iters=2, gamma=0.99, lam=0.95, use_graphs=False)
    tr = VecTrainer(cfg, device=cuda)
    p0 = tr.pi.params.clone()
    tr.train_epoch()
    torch.cuda.synchronize()
    m = tr.metrics()
    assert torch.isfinite(tr.pi.params).all() and not torch.equal(p0, tr.pi.params)
    assert math.isfinite(m["LossPi"]) and math.isfinite(m["LossV"])
    cols = torch.randperm(N, generator=torch.Generator().manual_seed(1))[:32].to(cuda)
    rl = tr.rl
    a_ref, r_ref, _ = ref.gae_scan_tm_ref(tr.rew[:, cols].double().cpu(), tr.done[:, cols].double().cpu(),
                                          rl.val.view(T + 1, N)[:, cols].double().cpu().reshape(-1), 0.99, 0.95,
                                          rl.tval[:, cols].double().cpu())
    torch.testing.assert_close(rl.adv[:, cols].double().cpu(), a_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rl.ret[:, cols].double().cpu(), r_ref, rtol=1e-4, atol=1e-4)
    # the last env column's final observation sits past byte offset 2^31 of the obs buffer
    assert tr.obs.numel() * 4 > 2 ** 31 and torch.isfinite(tr.obs[T, N - 1]).all()
    del tr
    torch.cuda.empty_cache()
