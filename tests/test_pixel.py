"""Pixel A2C family on CPU: Nature-CNN spec / oracle, PongSynth numpy reference, the A2C
trainer (oracle path) and its DP gradient all-reduce over gloo (world 2)."""
import numpy as np
import pytest
import torch
import torch.distributed as dist

from relayrl_prototype_amd.envs.pong import PongRef, nhwc_to_s2d, s2d_to_nhwc
from relayrl_prototype_amd.models.nature_cnn import CNNSpec, a2c_loss, reference_forward


def test_cnn_spec_layout_and_forward():
    spec = CNNSpec(6)
    o = spec.offsets()
    assert o["w1"] == 0 and o["b1"] == 32 * 256 and o["P"] == spec.P
    assert spec.P == 8192 + 32 + 32768 + 64 + 36864 + 64 + 3136 * 512 + 512 + 6 * 512 + 6 + 512 + 1
    p = spec.init(0)
    assert torch.equal(p, spec.init(0)) and not torch.equal(p, spec.init(1))
    obs = torch.randint(0, 256, (3, 21, 21, 64), dtype=torch.uint8)
    logits, value, acts = reference_forward(spec, p, obs)
    # the NHWC form of the same frames gives the same outputs
    l_n, v_n, _ = reference_forward(spec, p, s2d_to_nhwc(obs).contiguous())
    assert torch.allclose(l_n, logits) and torch.allclose(v_n, value)
    assert logits.shape == (3, 6) and value.shape == (3,)
    assert [a.shape[1:] for a in acts[:3]] == [(32, 20, 20), (64, 9, 9), (64, 7, 7)] and acts[3].shape == (3, 512)
    # bf16 emulation stays close to fp32
    l2, v2, _ = reference_forward(spec, p, obs, emulate_bf16=True)
    assert torch.allclose(l2, logits, atol=5e-3) and torch.allclose(v2, value, rtol=5e-2, atol=5e-2)


def test_conv1_s2d_weight_order_roundtrip():
    from relayrl_prototype_amd.models.nature_cnn import conv1_khkwc_to_s2d, conv1_s2d_to_khkwc

    w = torch.randn(32, 8, 8, 4)
    assert torch.equal(conv1_s2d_to_khkwc(conv1_khkwc_to_s2d(w)), w)
    # 8x8/4 conv on NHWC == 2x2/1 conv on the s2d input with s2d-ordered weights
    x = torch.rand(2, 84, 84, 4)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), stride=4)
    xs = nhwc_to_s2d(x).permute(0, 3, 1, 2)
    ws = conv1_khkwc_to_s2d(w).permute(0, 3, 1, 2)
    assert torch.allclose(torch.nn.functional.conv2d(xs, ws, stride=1), ref, atol=1e-4)


def test_a2c_loss_gradients_finite():
    spec = CNNSpec(6)
    p = spec.init(0).requires_grad_(True)
    obs = torch.randint(0, 256, (4, 21, 21, 64), dtype=torch.uint8)
    lg, v, _ = reference_forward(spec, p, obs)
    loss, pg, vf, ent = a2c_loss(lg, v, torch.tensor([0, 1, 2, 5]), torch.randn(4), torch.randn(4), 0.5, 0.01)
    loss.backward()
    assert torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0
    assert abs(ent.item() - np.log(6)) < 1e-2  # near-uniform initial policy (0.01 gain)


def test_pong_reference_dynamics():
    env = PongRef(16, seed=3, max_steps=400)
    obs = env.reset()
    assert obs.shape == (16, 21, 21, 64) and obs.dtype == np.uint8
    assert np.array_equal(nhwc_to_s2d(s2d_to_nhwc(obs)), obs)
    obs = s2d_to_nhwc(obs)
    assert (obs[:, 0] == 100).all() and (obs[:, 83] == 100).all()  # walls
    assert (obs == 255).any()  # paddles / ball drawn
    rng = np.random.default_rng(0)
    total = np.zeros(16)
    dones = 0
    for _ in range(450):
        r, d, fr, fl = env.step(rng.integers(0, 6, 16))
        total += r
        dones += d.sum()
        assert set(np.unique(r)).issubset({-1.0, 0.0, 1.0})
    assert (total < 0).sum() >= 8  # a random paddle loses points to the tracking opponent
    assert dones >= 16  # max_steps truncation (or 21 points) ended every env at least once
    o = env.render_nhwc()
    # the newest frame's ball is drawn where the state says
    bx, by = env.s[0, 16 + 12], env.s[0, 16 + 13]
    if 0 <= bx < 83 and 2 <= by < 81:
        assert o[0, int(by + 0.5), int(bx + 0.5), 3] == 255


def test_pixel_trainer_cpu_updates():
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    tr = PixelA2CTrainer(PixelA2CConfig(num_envs=4, rollout_len=3, seed=1), device="cpu")
    p0 = tr.params.detach().clone()
    for _ in range(2):
        st = tr.train_epoch()
    assert not torch.equal(p0, tr.params.detach())
    m = tr.metrics()
    assert m["EnvSteps"] == 2 * 4 * 3 and np.isfinite(m["LossPi"]) and np.isfinite(m["LossV"])
    assert abs(m["Entropy"] - np.log(6)) < 0.05


def _worker_pixel_dp(rank, world, port, q):
    try:
        from test_distributed import _init

        comm = _init(rank, world, port)
        from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

        tr = PixelA2CTrainer(PixelA2CConfig(num_envs=2, rollout_len=2, seed=5), comm, device="cpu")
        tr.train_epoch()
        p = tr.params.detach().clone()
        gathered = [torch.zeros_like(p) for _ in range(world)]
        dist.all_gather(gathered, p)
        # different env streams per rank, yet identical weights after the all-reduced step
        q.put((rank, all(torch.equal(gathered[0], x) for x in gathered), float(tr.rew.abs().sum())))
        dist.destroy_process_group()
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc(), None))


def test_pixel_trainer_dp_gloo():
    from test_distributed import _run

    res = _run(_worker_pixel_dp)
    for rank, ok, _ in res:
        assert ok is True, (rank, ok)


def test_frame_ring_layout_gives_the_s2d_observation():
    """FrameRing's store layout (one s2d frame [21][21][4][4] per slot and env) and frame rows:
    gathering frames 0..3 of PongRef's stack through fidx reproduces its s2d observation, and a
    reset env's clamped rows (all pointing at one frame) give its 4 identical frames."""
    from relayrl_prototype_amd.envs.pong import VALID, FrameRing

    N = 5
    env = PongRef(N, seed=3, max_steps=4)
    env.reset()
    for _ in range(3):
        env.step(np.random.default_rng(0).integers(0, 6, N))
    stack = env.render_nhwc()                       # [N, 84, 84, 4]
    ring = FrameRing(N, 7, "cpu")
    fr = ring.frames.view(7, N, 21, 4, 21, 4)      # [slot][env][a][dy][b][dx] as an image view
    for f in range(4):                              # frame f of the stack into slot f
        img = torch.from_numpy(stack[..., f].copy()).view(N, 21, 4, 21, 4)
        fr[f].copy_(img)
    # the store is s2d per frame: [slot][env][a][b][dy][dx]
    ring.frames.copy_(fr.permute(0, 1, 2, 4, 3, 5).contiguous().view(-1))
    fidx = torch.tensor([[f * N + e for f in range(4)] for e in range(N)], dtype=torch.int32)
    assert torch.equal(ring.gather_s2d(fidx), torch.from_numpy(env.render()))
    # the oracle's count of distinct frames: 1 after a reset, +1 per step up to 4
    assert set(np.unique(env.s[:, VALID]).tolist()) <= {1.0, 2.0, 3.0, 4.0}
    same = torch.full((1, 4), 2 * N, dtype=torch.int32)
    o = ring.gather_s2d(same).view(1, 21, 21, 16, 4)
    assert all(torch.equal(o[..., f], o[..., 0]) for f in range(4))
