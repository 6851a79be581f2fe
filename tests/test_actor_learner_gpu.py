"""Learner-shard layout on the GPU: the K-block time-major scan and the actor-learner
engine on cuda:0 (multi-rank RCCL runs need >1 GPU and are exercised by the driver's
scaling bench; the topology / lag logic is covered over gloo in test_distributed.py)."""
import pytest
import torch

from relayrl_prototype_amd.ops import gae_scan_tm
from relayrl_prototype_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,T,N", [(2, 16, 300), (3, 64, 1000), (8, 5, 33)])
def test_gae_scan_blocks(cuda, K, T, N):
    torch.manual_seed(K * T + N)
    rew = torch.randn(K, T, N)
    u = torch.rand(K, T, N)
    done = torch.where(u < 0.04, torch.ones_like(u), torch.where(u < 0.06, torch.full_like(u, 2.0),
                                                                  torch.zeros_like(u)))
    val = torch.randn(K * T * N + K * N)
    tval = torch.randn(K, T, N)
    a_r, r_r, s_r = ref.gae_scan_tm_ref(rew, done, val, 0.98, 0.97, tval)
    a_g, r_g, s_g = gae_scan_tm(rew.to(cuda), done.to(cuda), val.to(cuda), 0.98, 0.97, tval=tval.to(cuda))
    torch.testing.assert_close(a_g.cpu(), a_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(r_g.cpu(), r_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(s_g.cpu(), s_r, rtol=1e-3, atol=1e-2)


def test_rollout_learner_blocks_match_oracle(cuda):
    """K = 3 actor blocks through the HIP learner == the same batch through the CPU oracle."""
    from relayrl_prototype_amd.algorithms.learner import PGLearner
    from relayrl_prototype_amd.runtime.rollout_learn import RolloutLearner

    K, T, N, D, A = 3, 16, 64, 4, 2
    g = torch.Generator().manual_seed(0)
    obs = torch.randn(K * T * N + K * N, D, generator=g)
    act = torch.randint(0, A, (K, T, N), generator=g, dtype=torch.int32)
    rew = torch.rand(K, T, N, generator=g)
    u = torch.rand(K, T, N, generator=g)
    done = torch.where(u < 0.05, torch.ones_like(u), torch.where(u < 0.07, torch.full_like(u, 2.0),
                                                                  torch.zeros_like(u)))
    logp = -torch.rand(K, T, N, generator=g)
    tobs = torch.randn(K, T, N, D, generator=g)
    out = []
    for dev in ("cpu", cuda):
        lr = PGLearner("reinforce", D, A, 128, True, True, 3e-4, 1e-3, 3, device=dev, seed=1, use_graphs=False)
        rl = RolloutLearner(lr, T, N, 0.98, 0.97, blocks=K)
        rl.learn(obs.to(dev), act.to(dev), rew.to(dev), done.to(dev), logp.to(dev), tobs=tobs.to(dev))
        out.append((lr.pi.params.cpu(), lr.vf.params.cpu(), rl.ret.cpu()))
    torch.testing.assert_close(out[1][2], out[0][2], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out[1][0], out[0][0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(out[1][1], out[0][1], rtol=1e-4, atol=1e-5)


def test_actor_learner_colocated_gpu(cuda):
    from relayrl_prototype_amd.runtime.actor_learner import ActorLearner, ActorLearnerConfig

    al = ActorLearner(ActorLearnerConfig(env="LunarLanderSynth-v0", num_envs=512, rollout_len=32,
                                         train_vf_iters=4, verify_versions=True), device=cuda)
    assert al.actor.kind == "device" and al.topo.K == 1
    p0 = al.learner.pi.params.clone()
    for _ in range(3):
        al.step()
    al.finish()
    m = al.metrics()
    assert m["EnvSteps"] == 3 * 32 * 512 and m["ActorVersions"] == [2]
    assert torch.isfinite(al.learner.pi.params).all() and not torch.equal(p0, al.learner.pi.params)
    assert torch.equal(al.actor.params, al.learner.pi.params)


def test_actor_learner_colocated_continuous_device_env(cuda):
    """HalfCheetahSynth under the actor-learner topology rolls out on the DEVICE (the
    Gaussian rollout_cont kernel), not on host threads."""
    from relayrl_prototype_amd.runtime.actor_learner import ActorLearner, ActorLearnerConfig

    al = ActorLearner(ActorLearnerConfig(env="HalfCheetahSynth-v0", algo="ppo", num_envs=1024, rollout_len=32,
                                         train_vf_iters=3, train_pi_iters=3, verify_versions=True,
                                         phase_timing=True), device=cuda)
    assert al.actor.kind == "device" and al.continuous and al.topo.K == 1
    p0 = al.learner.pi.params.clone()
    for _ in range(3):
        al.step()
    al.finish()
    m = al.metrics()
    assert m["EnvSteps"] == 3 * 32 * 1024 and m["ActorVersions"] == [2]
    assert m["RolloutMs"] > 0 and m["LearnMs"] > 0  # phase columns
    assert torch.isfinite(al.learner.pi.params).all() and not torch.equal(p0, al.learner.pi.params)
    assert al.b_act.dtype == torch.float32 and al.b_act.shape[-1] == 6


def test_grad_chunks_equal_one_launch(cuda, monkeypatch):
    """Batches past GRAD_CHUNK_ROWS are launched in chunks whose slabs sit back to back; the
    summed gradient equals the one-launch gradient (fp32 summation order aside)."""
    from relayrl_prototype_amd.ops import GradHead, mlp, MLPSpec, mlp_grad, reduce_slabs

    g = torch.Generator().manual_seed(3)
    B, D = 70_000, 17
    X = torch.randn(B, D, generator=g).to(cuda)
    ret = torch.randn(B, generator=g).to(cuda)
    vp = MLPSpec(D, 128, 1).init(g).to(cuda)
    one = reduce_slabs(mlp_grad(GradHead.VALUE_MSE, vp, X, 1, 128, ret=ret, inv_B=1.0 / B)[0])
    monkeypatch.setattr(mlp, "GRAD_CHUNK_ROWS", 16_384)
    assert len(mlp.grad_chunks(B)) == 5
    slab, ls = mlp_grad(GradHead.VALUE_MSE, vp, X, 1, 128, ret=ret, inv_B=1.0 / B)
    assert slab.shape[0] == mlp.grad_slabs(B, cuda)
    chunked = reduce_slabs(slab)
    torch.testing.assert_close(chunked, one, rtol=1e-4, atol=1e-6)
    assert int(ls[:, 5].sum().item()) == B  # every row counted once
