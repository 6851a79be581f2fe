"""Pixel-model HIP kernels (csrc/kernels/cnn.hip, pong.hip) against PyTorch fp32 oracles.

bf16 operands: the oracle rounds weights / inputs / stored activations to bf16 where the
kernels do and computes in fp32, so the remaining difference is accumulation order
(and bf16 rounding of gradients at layer boundaries for the backward)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from relayrl_prototype_amd.models.nature_cnn import (CONVS, FC_IN, HIDDEN, CNNSpec, DeviceNatureCNN, a2c_loss,
                                                    conv1_khkwc_to_s2d, conv1_s2d_to_khkwc, obs_to_nchw,
                                                    reference_forward)

pytestmark = pytest.mark.gpu


def relerr(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _bf(x):
    return x.to(torch.bfloat16).float()


@pytest.mark.parametrize("N", [1, 7, 64])
def test_conv1_forward_s2d(cuda, N):
    from relayrl_prototype_amd.ops import hip

    h = hip()
    g = torch.Generator().manual_seed(N)
    x = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g)
    w = torch.randn(32, 8, 8, 4, generator=g) * 0.05
    b = torch.randn(32, generator=g) * 0.1
    y = torch.empty(N * 400 * 32, dtype=torch.bfloat16, device=cuda)
    h.conv_fwd(x.to(cuda), conv1_khkwc_to_s2d(w).contiguous().to(cuda).bfloat16().reshape(-1), b.to(cuda), y, N, 21,
               21, 64, 2, 2, 1, 32, True)
    ref = F.relu(F.conv2d(_bf(obs_to_nchw(x)), _bf(w).permute(0, 3, 1, 2), b, stride=4))
    assert relerr(y, ref.permute(0, 2, 3, 1).reshape(-1)) < 1e-2


@pytest.mark.parametrize("N", [1, 7, 64])
def test_conv1_forward_u8(cuda, N):
    from relayrl_prototype_amd.ops import hip

    h = hip()
    L = CONVS[0]
    g = torch.Generator().manual_seed(N)
    x = torch.randint(0, 256, (N, 84, 84, 4), dtype=torch.uint8, generator=g)
    w = torch.randn(L.cout, L.k, L.k, L.cin, generator=g) * 0.05
    b = torch.randn(L.cout, generator=g) * 0.1
    y = torch.empty(N * 400 * 32, dtype=torch.bfloat16, device=cuda)
    h.conv_fwd(x.to(cuda), w.to(cuda).bfloat16().reshape(-1), b.to(cuda), y, N, 84, 84, 4, 8, 8, 4, 32, True)
    ref = F.relu(F.conv2d(_bf(x.float() / 255).permute(0, 3, 1, 2), _bf(w).permute(0, 3, 1, 2), b, stride=4))
    ref = ref.permute(0, 2, 3, 1).reshape(-1)
    assert relerr(y, ref) < 1e-2


@pytest.mark.parametrize("li,N", [(1, 5), (2, 33), (1, 130), (1, 1100), (2, 700)])
def test_conv_forward_bf16(cuda, li, N):
    from relayrl_prototype_amd.ops import hip

    h = hip()
    L = CONVS[li]
    g = torch.Generator().manual_seed(li * 100 + N)
    x = _bf(torch.rand(N, L.hin, L.hin, L.cin, generator=g))
    w = torch.randn(L.cout, L.k, L.k, L.cin, generator=g) * 0.05
    b = torch.randn(L.cout, generator=g) * 0.1
    y = torch.empty(N * L.hout ** 2 * L.cout, dtype=torch.bfloat16, device=cuda)
    h.conv_fwd(x.to(cuda).bfloat16(), w.to(cuda).bfloat16().reshape(-1), b.to(cuda), y, N, L.hin, L.hin, L.cin, L.k,
               L.k, L.s, L.cout, True)
    ref = F.relu(F.conv2d(x.permute(0, 3, 1, 2), _bf(w).permute(0, 3, 1, 2), b, stride=L.s))
    assert relerr(y, ref.permute(0, 2, 3, 1).reshape(-1)) < 1e-2


@pytest.mark.parametrize("li,N", [(1, 6), (2, 19), (1, 900)])
def test_conv_dgrad_col2im_and_wgrad(cuda, li, N):
    """dX (masked by the input activation) and dW / db of a conv vs autograd."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    L = CONVS[li]
    g = torch.Generator().manual_seed(7 + li + N)
    x = _bf(F.relu(torch.randn(N, L.hin, L.hin, L.cin, generator=g)))  # post-ReLU input (mask source)
    w = _bf(torch.randn(L.cout, L.k, L.k, L.cin, generator=g) * 0.05)
    dy = _bf(torch.randn(N, L.hout, L.hout, L.cout, generator=g))
    xt = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    wt = w.permute(0, 3, 1, 2).clone().requires_grad_(True)
    out = F.conv2d(xt, wt, stride=L.s)
    out.backward(dy.permute(0, 3, 1, 2))
    dx_ref = (xt.grad * (xt > 0)).permute(0, 2, 3, 1).reshape(-1)
    dw_ref = wt.grad.permute(0, 2, 3, 1).reshape(-1)
    M, K = N * L.hout ** 2, L.K
    dcol = torch.empty(M * K, dtype=torch.bfloat16, device=cuda)
    dyd = dy.to(cuda).bfloat16().reshape(-1)
    wd = w.to(cuda).bfloat16().reshape(-1)
    xd = x.to(cuda).bfloat16().reshape(-1)
    h.gemm_dgrad(dyd, wd, None, dcol, M, L.cout, K)
    dx = torch.empty(N * L.hin ** 2 * L.cin, dtype=torch.bfloat16, device=cuda)
    h.col2im_mask(dcol, xd, dx, N, L.hin, L.hin, L.cin, L.k, L.k, L.s)
    assert relerr(dx, dx_ref) < 2e-2
    dx2 = torch.full_like(dx, float("nan"))
    assert h.conv_dgrad(dyd, wd, xd, dx2, N, L.hin, L.hin, L.cin, L.k, L.k, L.s, L.cout)  # implicit path exists
    assert relerr(dx2, dx_ref) < 1e-2
    for splits in (1, 7):
        s = int(h.gemm_splits(M, splits))
        part = torch.empty(s * L.cout * K, device=cuda)
        bsp = torch.empty(s * L.cout, device=cuda)
        s2 = int(h.conv_wgrad(dyd, xd, part, splits, N, L.hin, L.hin, L.cin, L.k, L.k, L.s, L.cout, bsp))
        assert s2 == s
        dw = torch.empty(L.cout * K, device=cuda)
        h.sum_splits(part, s, L.cout * K, dw)
        assert relerr(dw, dw_ref) < 1e-2, splits
        dbs = torch.empty(L.cout, device=cuda)
        h.sum_splits(bsp, s, L.cout, dbs)  # bias partials requested from the generic path (column sums)
        assert relerr(dbs, dy.reshape(-1, L.cout).sum(0)) < 1e-4
    bp = torch.empty(3 * L.cout, device=cuda)
    h.colsum(dyd, M, L.cout, bp, 3)
    db = torch.empty(L.cout, device=cuda)
    h.sum_splits(bp, 3, L.cout, db)
    assert relerr(db, dy.reshape(-1, L.cout).sum(0)) < 1e-4


@pytest.mark.parametrize("N,splits", [(9, 16), (300, 64), (5, 256)])
def test_conv1_wgrad_from_s2d_frames(cuda, N, splits):
    """Streaming conv1 weight-gradient kernel (one pass over frames + dY) vs autograd;
    (5, 256): more partial slabs than images, the idle workgroups must write zeros."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    g = torch.Generator().manual_seed(12)
    x = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g)
    dy = _bf(torch.randn(N, 20, 20, 32, generator=g))
    wt = torch.zeros(32, 4, 8, 8, requires_grad=True)
    F.conv2d(_bf(obs_to_nchw(x)), wt, stride=4).backward(dy.permute(0, 3, 1, 2))
    dw_ref = conv1_khkwc_to_s2d(wt.grad.permute(0, 2, 3, 1)).reshape(-1)
    M = N * 400
    s = int(h.gemm_splits(M, splits))
    part = torch.full((s * 32 * 256,), float("nan"), device=cuda)
    bpart = torch.full((s * 32,), float("nan"), device=cuda)
    h.conv_wgrad(dy.to(cuda).bfloat16().reshape(-1), x.to(cuda), part, splits, N, 21, 21, 64, 2, 2, 1, 32, bpart)
    dw = torch.empty(32 * 256, device=cuda)
    h.sum_splits(part, s, 32 * 256, dw)
    assert relerr(dw, dw_ref) < 1e-2
    db = torch.empty(32, device=cuda)
    h.sum_splits(bpart, s, 32, db)  # fused bias gradient
    assert relerr(db, dy.reshape(-1, 32).sum(0)) < 1e-4


def test_conv1_wgrad_from_frames(cuda):
    from relayrl_prototype_amd.ops import hip

    h = hip()
    L = CONVS[0]
    N = 9
    g = torch.Generator().manual_seed(11)
    x = torch.randint(0, 256, (N, 84, 84, 4), dtype=torch.uint8, generator=g)
    dy = _bf(torch.randn(N, 20, 20, 32, generator=g))
    xt = _bf(x.float() / 255).permute(0, 3, 1, 2)
    wt = torch.zeros(32, 4, 8, 8, requires_grad=True)
    F.conv2d(xt, wt, stride=4).backward(dy.permute(0, 3, 1, 2))
    dw_ref = wt.grad.permute(0, 2, 3, 1).reshape(-1)
    M = N * 400
    s = int(h.gemm_splits(M, 16))
    part = torch.empty(s * 32 * 256, device=cuda)
    h.conv_wgrad(dy.to(cuda).bfloat16().reshape(-1), x.to(cuda), part, 16, N, 84, 84, 4, 8, 8, 4, 32)
    dw = torch.empty(32 * 256, device=cuda)
    h.sum_splits(part, s, 32 * 256, dw)
    assert relerr(dw, dw_ref) < 1e-2


def test_fc_dgrad_masked(cuda):
    from relayrl_prototype_amd.ops import hip

    h = hip()
    B = 37
    g = torch.Generator().manual_seed(3)
    dh = _bf(torch.randn(B, HIDDEN, generator=g))
    w = _bf(torch.randn(HIDDEN, FC_IN, generator=g) * 0.02)
    a3 = _bf(F.relu(torch.randn(B, FC_IN, generator=g)))
    out = torch.empty(B * FC_IN, dtype=torch.bfloat16, device=cuda)
    h.gemm_dgrad(dh.to(cuda).bfloat16().reshape(-1), w.to(cuda).bfloat16().reshape(-1),
                 a3.to(cuda).bfloat16().reshape(-1), out, B, HIDDEN, FC_IN)
    assert relerr(out, ((dh @ w) * (a3 > 0)).reshape(-1)) < 1e-2


@pytest.mark.parametrize("B", [48, 50])  # 3-4 rows per wave in the head backward (next-row prefetch, tail)
@pytest.mark.parametrize("mfma", ["0", "1"])  # RRL_HEAD_MFMA: the fp32-MFMA head backward (partial last tile at 50)
def test_full_model_forward_backward_matches_autograd(cuda, B, mfma, monkeypatch):
    monkeypatch.setenv("RRL_HEAD_MFMA", mfma)
    spec = CNNSpec(6)
    params = spec.init(4)
    # larger head weights so the policy gradient is not negligible next to the value part
    o = spec.offsets()
    params[o["wpi"]:o["bpi"]] *= 50.0
    m = DeviceNatureCNN(spec, cuda, max_batch=B, params=params)
    g = torch.Generator().manual_seed(5)
    obs = torch.randint(0, 256, (B, 21, 21, 64), dtype=torch.uint8, generator=g)
    act = torch.randint(0, 6, (B,), dtype=torch.int32, generator=g)
    adv = torch.randn(B, generator=g)
    ret = torch.randn(B, generator=g)
    lg, val = m.logits(obs.to(cuda))
    pe = params.clone().requires_grad_(True)
    rl, rv, _ = reference_forward(spec, pe, obs, emulate_bf16=True)
    assert relerr(lg, rl.detach()) < 2e-2 and relerr(val, rv.detach()) < 2e-2
    m.forward(obs.to(cuda), 0)
    stats = m.backward(obs.to(cuda), act.to(cuda), adv.to(cuda), ret.to(cuda), 0.5, 0.01)
    loss, pg, vf, ent = a2c_loss(rl, rv, act, adv, ret, 0.5, 0.01)
    loss.backward()
    gd = m.grad.cpu()
    for name, (a, b) in {"conv1": (o["w1"], o["b1"]), "conv2": (o["w2"], o["b2"]), "conv3": (o["w3"], o["b3"]),
                         "fc": (o["wfc"], o["bfc"]), "head": (o["head"], o["P"])}.items():
        e = relerr(gd[a:b], pe.grad[a:b])
        assert e < 5e-2, (name, e)
        # biases separately (a wrong bias partial hides inside the weight block's norm)
        if name.startswith("conv") or name == "fc":
            nb = HIDDEN if name == "fc" else CONVS[int(name[-1]) - 1].cout
            eb = relerr(gd[b:b + nb], pe.grad[b:b + nb])
            assert eb < 5e-2, (name, "bias", eb)
    st = stats.sum(0).cpu()
    assert abs(st[3].item() - B) < 1e-3
    assert abs(st[0].item() / B - pg.item()) < 2e-2 * max(1.0, abs(pg.item()))
    assert abs(st[2].item() / B - ent.item()) < 1e-2


def test_adam_clip_matches_torch(cuda):
    from relayrl_prototype_amd.ops import hip

    h = hip()
    n = 10007
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * 3 for _ in range(3)]
    p = p0.clone().to(cuda)
    mm = torch.zeros(n, device=cuda)
    vv = torch.zeros(n, device=cuda)
    sh = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    work = torch.empty(64, device=cuda)
    nsq = torch.empty(1, device=cuda)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-3, eps=1e-5)
    for i, gr in enumerate(grads, 1):
        gd = gr.to(cuda)
        h.sumsq(gd, work, nsq)
        h.adam_clip(p, mm, vv, gd, sh, nsq, 0.5, 1e-3, 0.9, 0.999, 1e-5, i)
        ref.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_([ref], 0.5)
        opt.step()
    assert torch.allclose(p.cpu(), ref.detach(), atol=1e-5)
    assert torch.equal(sh.cpu(), p.cpu().bfloat16())


def test_adam_clip_norm_parts_equals_two_launch_norm(cuda):
    """The clip + Adam launch reducing the sum-of-squares partials itself (norm_parts) gives
    bitwise the update of the separate sumsq -> sum_small -> adam_clip sequence."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    n = 300007
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g).to(cuda)
    gr = (torch.randn(n, generator=g) * 5).to(cuda)
    outs = []
    for fused in (False, True):
        p, mm, vv = p0.clone(), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
        sh = torch.empty(n, dtype=torch.bfloat16, device=cuda)
        work = torch.empty(1024, device=cuda)
        nsq = torch.empty(1, device=cuda)
        for i in range(1, 4):
            if fused:
                parts = int(h.sumsq_partial(gr, work))
                h.adam_clip(p, mm, vv, gr, sh, work, 0.5, 1e-3, 0.9, 0.999, 1e-5, i, norm_parts=parts)
            else:
                h.sumsq(gr, work, nsq)
                h.adam_clip(p, mm, vv, gr, sh, nsq, 0.5, 1e-3, 0.9, 0.999, 1e-5, i)
        torch.cuda.synchronize()
        outs.append((p, mm, vv, sh))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_head_sampling_distribution(cuda):
    spec = CNNSpec(6)
    B = 4096
    params = spec.init(2)
    o = spec.offsets()
    params[o["wpi"]:o["bpi"]] *= 80.0
    m = DeviceNatureCNN(spec, cuda, max_batch=B, params=params)
    obs = torch.randint(0, 256, (1, 21, 21, 64), dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
    obs = obs.expand(B, 21, 21, 64).contiguous().to(cuda)
    act = torch.empty(B, dtype=torch.int32, device=cuda)
    logp = torch.empty(B, device=cuda)
    val = torch.empty(B, device=cuda)
    m.act(obs, 0, act, logp, val, seed=9, step=3)
    lg, _ = m.logits(obs[:1])
    p = torch.softmax(lg[0].cpu(), -1)
    freq = torch.bincount(act.cpu().long(), minlength=6).float() / B
    assert (freq - p).abs().max() < 0.03
    # the batch-4096 and batch-1 forwards take different fc schedules (split-K for tiny
    # batches), so the bf16-rounded hidden units can differ in the last bit: ~1e-4 in logp
    assert torch.allclose(logp.cpu(), torch.log(p)[act.cpu().long()], atol=1e-3)


def test_device_pong_matches_reference(cuda):
    from relayrl_prototype_amd.envs.pong import DevicePong, PongRef

    N, steps = 64, 60
    ref = PongRef(N, seed=21, max_steps=50)
    dev = DevicePong(N, cuda, seed=21, max_steps=50)
    obs = torch.empty(N, 21, 21, 64, dtype=torch.uint8, device=cuda)
    o_ref = ref.reset()
    dev.reset(obs)
    assert (obs.cpu().numpy() != o_ref).mean() < 1e-3
    rng = np.random.default_rng(1)
    mism = 0
    for _ in range(steps):
        a = rng.integers(0, 6, N).astype(np.int32)
        r, d, fr, fl = ref.step(a)
        rd, dd = dev.step(torch.from_numpy(a).to(cuda), obs)
        mism += int((dd.cpu().numpy() != d).sum() + (rd.cpu().numpy() != r).sum())
    # fp32 contraction differences may flip a rare paddle-edge contact; allow a couple
    assert mism <= 2, mism
    st = dev.state.view(N, -1).cpu().numpy()
    close = np.all(np.abs(st[:, :10] - ref.s[:, :10]) < 2e-3, axis=1)
    assert close.mean() >= 0.95, close.mean()
    assert (obs.cpu().numpy() != ref.render()).mean() < 5e-3


def test_pixel_trainer_gpu_runs(cuda):
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    tr = PixelA2CTrainer(PixelA2CConfig(num_envs=64, rollout_len=5, seed=2), device=cuda)
    p0 = tr.model.params.clone()
    for _ in range(3):
        tr.train_epoch()
    torch.cuda.synchronize()
    m = tr.metrics()
    assert not torch.equal(p0, tr.model.params)
    assert torch.isfinite(tr.model.params).all()
    assert np.isfinite(m["LossPi"]) and np.isfinite(m["LossV"]) and abs(m["Entropy"] - np.log(6)) < 0.1
    assert m["EnvSteps"] == 3 * 64 * 5


@pytest.mark.parametrize("B", [37, 512])
def test_fc_forward_splitk_matches_direct(cuda, B):
    from relayrl_prototype_amd.ops import hip

    h = hip()
    g = torch.Generator().manual_seed(B)
    x = _bf(F.relu(torch.randn(B, FC_IN, generator=g)))
    w = _bf(torch.randn(HIDDEN, FC_IN, generator=g) * 0.02)
    b = torch.randn(HIDDEN, generator=g) * 0.1
    xd, wd, bd = x.to(cuda).bfloat16().reshape(-1), w.to(cuda).bfloat16().reshape(-1), b.to(cuda)
    y1 = torch.empty(B * HIDDEN, dtype=torch.bfloat16, device=cuda)
    y2 = torch.empty_like(y1)
    h.conv_fwd(xd, wd, bd, y1, B, 1, 1, FC_IN, 1, 1, 1, HIDDEN, True)
    work = torch.empty(16 * B * HIDDEN, device=cuda)
    h.conv_fwd(xd, wd, bd, y2, B, 1, 1, FC_IN, 1, 1, 1, HIDDEN, True, work)
    ref = F.relu(x @ w.t() + b).reshape(-1)
    assert relerr(y1, ref) < 1e-2 and relerr(y2, ref) < 1e-2


def _dp_worker(rank, world, port, q):
    import os

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), RRL_DIST_BACKEND="gloo", RRL_FORCE_DEVICE="0")
        import torch.distributed as dist

        from relayrl_prototype_amd.parallel.comm import init_distributed

        comm = init_distributed()
        dev = torch.device("cuda", 0)
        spec = CNNSpec(6)
        B = 16
        m = DeviceNatureCNN(spec, dev, max_batch=B, params=spec.init(3))
        grads = []
        for r in range(world):  # every rank computes every rank's local gradient (oracle)
            g = torch.Generator().manual_seed(100 + r)
            obs = torch.randint(0, 256, (B, 21, 21, 64), dtype=torch.uint8, generator=g).to(dev)
            act = torch.randint(0, 6, (B,), dtype=torch.int32, generator=g).to(dev)
            adv, ret = torch.randn(B, generator=g).to(dev), torch.randn(B, generator=g).to(dev)
            m.forward(obs, 0)
            m.backward(obs, act, adv, ret, 0.5, 0.01)
            grads.append(m.grad.clone())
            if r == rank:
                mine = (obs, act, adv, ret)
        m.forward(mine[0], 0)
        m.backward(*mine, 0.5, 0.01, comm=comm)  # bucketed, overlapped all-reduce
        expect = sum(grads) / world
        err = ((m.grad - expect).norm() / expect.norm()).item()
        q.put((rank, err))
        dist.destroy_process_group()
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc()))


def test_cnn_dp_overlapped_allreduce_matches_mean_gradient(cuda):
    """Two ranks (gloo, sharing the one GPU): the overlapped two-bucket all-reduce equals the
    mean of the per-rank gradients."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    for rank, err in res:
        assert isinstance(err, float) and err < 1e-5, (rank, err)


def test_pixel_trainer_graph_replay_matches_eager(cuda):
    """The captured update (device RNG / Adam counters) reproduces the eager updates exactly."""
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    cfg = dict(num_envs=32, rollout_len=4, seed=9)
    a = PixelA2CTrainer(PixelA2CConfig(use_graphs=True, **cfg), device=cuda)
    b = PixelA2CTrainer(PixelA2CConfig(use_graphs=False, **cfg), device=cuda)
    for _ in range(4):  # eager warm-up, capture+replay, 2 replays
        a.train_epoch()
        b.train_epoch()
    torch.cuda.synchronize()
    assert a._graph is not None and b._graph is None
    assert torch.equal(a.act, b.act) and torch.equal(a.obs, b.obs)
    torch.testing.assert_close(a.model.params, b.model.params, rtol=0, atol=0)
    assert int(a.model.step_t.item()) == 4 and a.env.step_count == b.env.step_count


@pytest.mark.parametrize("splits,n", [(256, 3591), (3, 7), (17, 4096)])
def test_sum_splits_matches_torch(cuda, splits, n):
    """Split-slab reduction, including the unaligned / odd-length path (A2C head: n = 3591)."""
    from relayrl_prototype_amd.ops import hip

    g = torch.Generator().manual_seed(splits + n)
    part = torch.randn(splits, n, generator=g)
    out = torch.empty(n, device=cuda)
    hip().sum_splits(part.to(cuda).reshape(-1), splits, n, out)
    torch.testing.assert_close(out.cpu(), part.sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("variant", [128, 64], ids=["8wave", "16wave"])
@pytest.mark.parametrize("N", [1, 5, 300, 2048])
def test_fused_conv_stack_matches_per_layer_kernels(cuda, N, variant):
    """conv_stack_fwd (conv1 -> conv2 -> conv3 in one launch, cnn_fused.hip; the 8-wave kernel and
    the 16-wave three-stage pipeline) against the per-layer kernels it replaces (equal up to fma
    contraction / summation order) and the bf16-emulating fp32 oracle."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    spec = CNNSpec()
    o = spec.offsets()
    g = torch.Generator().manual_seed(N)
    params = spec.init(N).to(cuda)
    params += 0.01 * torch.randn(params.shape, generator=g).to(cuda)  # non-zero biases
    sh = params.bfloat16()
    x = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    outs = []
    for fused in (True, False):
        a1 = torch.full((N * 400 * 32,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a2 = torch.full((N * 81 * 64,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a3 = torch.full((N * FC_IN,), float("nan"), dtype=torch.bfloat16, device=cuda)
        if fused:
            h.conv_stack_fwd(x, sh[o["w1"]:o["b1"]], params[o["b1"]:o["b1"] + 32], sh[o["w2"]:o["b2"]],
                             params[o["b2"]:o["b2"] + 64], sh[o["w3"]:o["b3"]], params[o["b3"]:o["b3"] + 64], a1, a2,
                             a3, N, probe=variant)
        else:
            from relayrl_prototype_amd.models.nature_cnn import S2D

            src = x
            for i, (L, y) in enumerate(zip((S2D,) + CONVS[1:], (a1, a2, a3)), 1):
                h.conv_fwd(src, sh[o[f"w{i}"]:o[f"b{i}"]], params[o[f"b{i}"]:o[f"b{i}"] + L.cout], y, N, L.hin,
                           L.hin, L.cin, L.k, L.k, L.s, L.cout, True)
                src = y
        torch.cuda.synchronize()
        outs.append((a1, a2, a3))
    for f, r in zip(outs[0], outs[1]):
        assert torch.isfinite(f.float()).all()
        # equal up to bf16 rounding flips where an fma contraction differs
        assert relerr(f, r) < 2e-3
    _, _, acts = reference_forward(spec, params.cpu(), x.cpu(), emulate_bf16=True)
    for dev_a, ref_a in zip(outs[0], acts[:3]):
        assert relerr(dev_a, ref_a.permute(0, 2, 3, 1).reshape(-1)) < 1e-2


@pytest.mark.parametrize("B", [3, 300, 1500])
def test_fused_conv_backward_matches_per_layer(cuda, B, monkeypatch):
    """The fused conv3 backward (dgrad + wgrad + bias in one pass, cnn_fused.hip) against the
    per-layer kernels on the same stored activations: every parameter gradient.  The fused side's
    forward is the 8-wave kernel, whose conv1 k-order is the per-layer kernel's (the 16-wave
    forward sums conv1 in another order: a few bf16 activations flip, and with them ReLU masks)."""
    monkeypatch.setenv("RRL_CNN_FWD_LAYOUT", "128")
    spec = CNNSpec(6)
    o = spec.offsets()
    params = spec.init(7)
    params[o["wpi"]:o["bpi"]] *= 50.0
    g = torch.Generator().manual_seed(B)
    obs = torch.randint(0, 256, (B, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    act = torch.randint(0, 6, (B,), dtype=torch.int32, generator=g).to(cuda)
    adv = torch.randn(B, generator=g).to(cuda)
    ret = torch.randn(B, generator=g).to(cuda)
    grads = []
    for fused in (True, False):
        m = DeviceNatureCNN(spec, cuda, max_batch=B, params=params)
        m.fused_convs = fused
        m.forward(obs, 0)
        m.grad.fill_(float("nan"))
        m.backward(obs, act, adv, ret, 0.5, 0.01)
        torch.cuda.synchronize()
        grads.append(m.grad.clone())
    gf, gr = grads
    assert torch.isfinite(gf).all()
    for name, (a, b) in {"conv1": (o["w1"], o["b1"]), "conv2": (o["w2"], o["b2"]), "conv3": (o["w3"], o["b3"]),
                         "fc": (o["wfc"], o["bfc"]), "head": (o["head"], o["P"])}.items():
        assert relerr(gf[a:b], gr[a:b]) < 1e-4, name
    for i, L in enumerate(CONVS, 1):
        b0 = o[f"b{i}"]
        assert relerr(gf[b0:b0 + L.cout], gr[b0:b0 + L.cout]) < 1e-4, f"b{i}"


@pytest.mark.parametrize("li,N,grid,staged", [(1, 3, 3, 1), (1, 70, 16, 1), (1, 70, 16, 0), (1, 70, 16, 2),
                                              (2, 5, 5, 1), (2, 300, 64, 1)])
def test_fused_conv_bwd_kernels_match_autograd(cuda, li, N, grid, staged):
    """conv2_bwd / conv3_bwd (cnn_fused.hip) against fp32 autograd on the same bf16 operands:
    masked data gradient, weight-gradient partials (summed over workgroups), bias partials."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    L = CONVS[li]
    g = torch.Generator().manual_seed(li * 1000 + N)
    x = _bf(torch.relu(torch.randn(N, L.hin, L.hin, L.cin, generator=g)))  # post-ReLU input (zeros = mask)
    w = _bf(torch.randn(L.cout, L.k, L.k, L.cin, generator=g) * 0.05)
    dy = _bf(torch.randn(N, L.hout, L.hout, L.cout, generator=g))
    xd, wd, dyd = x.to(cuda).bfloat16(), w.to(cuda).bfloat16(), dy.to(cuda).bfloat16()
    dx = torch.full((N * L.hin * L.hin * L.cin,), float("nan"), dtype=torch.bfloat16, device=cuda)
    part = torch.full((grid * L.cout * L.K,), float("nan"), device=cuda)
    bpart = torch.full((grid * 512,), float("nan"), device=cuda)
    if li == 1:
        h.conv2_bwd(dyd.reshape(-1), wd.reshape(-1), xd.reshape(-1), dx, part, bpart, N, grid, staged=staged)
    else:
        h.conv3_bwd(dyd.reshape(-1), wd.reshape(-1), xd.reshape(-1), dx, part, bpart, N, grid)
    torch.cuda.synchronize()
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    wr = w.permute(0, 3, 1, 2).clone().requires_grad_(True)
    y = F.conv2d(xr, wr, stride=L.s)
    y.backward(dy.permute(0, 3, 1, 2))
    dx_ref = (xr.grad * (xr > 0)).permute(0, 2, 3, 1).reshape(-1)
    dw_ref = wr.grad.permute(0, 2, 3, 1).reshape(-1)
    db_ref = dy.sum((0, 1, 2))
    dxg = dx.float().cpu()
    assert torch.isfinite(dxg).all()
    assert relerr(dxg, dx_ref) < 1e-2
    dw = part.view(grid, -1).sum(0).cpu()
    assert relerr(dw, dw_ref) < 1e-3
    db = bpart[:grid * 64].view(grid, 64).sum(0).cpu()  # one 64-channel partial per workgroup
    assert relerr(db, db_ref) < 1e-3


@pytest.mark.parametrize("sp", ["0", "1"])  # RRL_CNN_WGRAD1_SETPRIO: the s_setprio form
@pytest.mark.parametrize("N,grid", [(1, 1), (9, 4), (300, 64)])
def test_conv1_wgrad8_matches_autograd(cuda, N, grid, sp, monkeypatch):
    """8-wave conv1 weight / bias gradient (cnn_fused.hip) vs fp32 autograd on the s2d frames."""
    from relayrl_prototype_amd.ops import hip

    monkeypatch.setenv("RRL_CNN_WGRAD1_SETPRIO", sp)
    h = hip()
    g = torch.Generator().manual_seed(N)
    x = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g)
    dy = _bf(torch.randn(N, 20, 20, 32, generator=g))
    part = torch.full((2 * grid * 32 * 256,), float("nan"), device=cuda)
    bpart = torch.full((2 * grid * 32,), float("nan"), device=cuda)
    ns = h.conv1_wgrad8(x.to(cuda), dy.to(cuda).bfloat16().reshape(-1), part, bpart, N, grid)
    assert ns == 2 * grid
    dw = part.view(ns, -1).sum(0).cpu()
    db = bpart.view(ns, 32).sum(0).cpu()
    w = torch.zeros(32, 8, 8, 4, requires_grad=True)
    y = F.conv2d(obs_to_nchw(x), w.permute(0, 3, 1, 2), stride=4)
    y.backward(dy.permute(0, 3, 1, 2))
    assert relerr(dw, conv1_khkwc_to_s2d(w.grad).reshape(-1)) < 1e-3
    assert relerr(db, dy.sum((0, 1, 2))) < 1e-3


# ----------------------------------------------------------------------------- fc.hip
@pytest.mark.parametrize("big", ["1", "0"])  # RRL_FC_BIG: persistent 256 x 128 tiles / 128 x 128 per workgroup
@pytest.mark.parametrize("M,N,K,splits", [(37, 512, 3136, 1), (300, 512, 3136, 4), (2048, 512, 3136, 4),
                                          (2048, 512, 3136, 8), (8192, 512, 3136, 2), (130, 3136, 512, 1),
                                          (5000, 3136, 512, 1), (64, 132, 128, 2)])
def test_fc_nt_part_matches_fp32(cuda, M, N, K, splits, big, monkeypatch):
    """DMA-staged NT GEMM (swizzled LDS images, 3-stage ring): the split-K partials sum to
    the fp32 product of the bf16 operands, for tile-ragged M and N; the persistent kernel walks
    several tiles per workgroup at (5000, 3136, 512) (500 tiles on 256 CUs)."""
    from relayrl_prototype_amd.ops import hip

    monkeypatch.setenv("RRL_FC_BIG", big)
    h = hip()
    g = torch.Generator().manual_seed(M + N + K)
    a = _bf(torch.randn(M, K, generator=g)).to(cuda)
    b = _bf(torch.randn(N, K, generator=g) * 0.05).to(cuda)
    part = torch.full((splits * M * N,), float("nan"), device=cuda)
    used = h.fc_nt_part(a.bfloat16().reshape(-1), b.bfloat16().reshape(-1), part, M, N, K, splits)
    assert 1 <= used <= splits
    got = part[:used * M * N].view(used, M, N).sum(0)
    ref = a.double() @ b.double().t()
    assert torch.isfinite(got).all()
    assert ((got.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5


@pytest.mark.parametrize("big", ["1", "0"])
@pytest.mark.parametrize("epi", ["0", "1"])  # RRL_FC_DIRECT_EPI: 0 = LDS-staged 16-byte epilogue, 1 = direct
@pytest.mark.parametrize("M", [37, 1000, 10240])
def test_fc_nt_mask_matches_fp32(cuda, M, epi, big, monkeypatch):
    from relayrl_prototype_amd.ops import hip

    if big == "1" and epi == "1":
        pytest.skip("the persistent kernel has one epilogue")
    monkeypatch.setenv("RRL_FC_DIRECT_EPI", epi)
    monkeypatch.setenv("RRL_FC_BIG", big)
    h = hip()
    g = torch.Generator().manual_seed(M)
    dh = _bf(torch.randn(M, HIDDEN, generator=g))
    w = _bf(torch.randn(HIDDEN, FC_IN, generator=g) * 0.02)
    a3 = _bf(F.relu(torch.randn(M, FC_IN, generator=g)))
    wt = torch.empty(FC_IN * HIDDEN, dtype=torch.bfloat16, device=cuda)
    h.transpose_bf16(w.to(cuda).bfloat16().reshape(-1), wt, HIDDEN, FC_IN)
    assert torch.equal(wt.view(FC_IN, HIDDEN).cpu().float(), w.t())
    out = torch.empty(M * FC_IN, dtype=torch.bfloat16, device=cuda)
    h.fc_nt_mask(dh.to(cuda).bfloat16().reshape(-1), wt, a3.to(cuda).bfloat16().reshape(-1), out, M, FC_IN, HIDDEN)
    ref = ((dh @ w) * (a3 > 0)).reshape(-1)
    assert relerr(out, ref) < 4e-3
    assert torch.equal((out.cpu().view(M, FC_IN) == 0) | (a3 > 0), torch.ones(M, FC_IN, dtype=torch.bool))


@pytest.mark.parametrize("B", [48, 2048])
def test_fc_head_fused_matches_separate(cuda, B, monkeypatch):
    """fc as split-K partials reduced inside the head launch (RRL_FC_NT=1, the default) vs the
    gemm_bf16.h fc + bias_act + head (RRL_FC_NT=0): same stored hidden units (to one bf16
    rounding), same value / log-prob, same sampled actions."""
    spec = CNNSpec(6)
    params = spec.init(7)
    o = spec.offsets()
    params[o["wpi"]:o["bpi"]] *= 30.0
    g = torch.Generator().manual_seed(B)
    obs = torch.randint(0, 256, (B, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("RRL_FC_NT", flag)
        m = DeviceNatureCNN(spec, cuda, max_batch=B, params=params)
        assert m.fc_nt == (flag == "1")
        act = torch.empty(B, dtype=torch.int32, device=cuda)
        logp = torch.empty(B, device=cuda)
        val = torch.empty(B, device=cuda)
        m.act(obs, 0, act, logp, val, seed=3, step=1)
        outs.append((act.cpu(), logp.cpu(), val.cpu(), m.hid[:B * HIDDEN].float().cpu()))
    (a1, l1, v1, h1), (a2, l2, v2, h2) = outs
    assert relerr(h1, h2) < 5e-3
    assert (h1 - h2).abs().max().item() <= 1e-2 * h2.abs().max().item()
    assert torch.allclose(v1, v2, atol=1e-3, rtol=1e-3)
    assert torch.allclose(l1, l2, atol=1e-3)
    assert (a1 != a2).float().mean().item() < 0.01


@pytest.mark.parametrize("big", ["1", "0"])
@pytest.mark.parametrize("R,I,J,splits", [(64, 512, 3136, 1), (640, 512, 3136, 5), (10240, 512, 3136, 5),
                                          (192, 136, 72, 2), (256, 4096, 3136, 1)])
def test_fc_tn_part_matches_fp32(cuda, R, I, J, splits, big, monkeypatch):
    """Weight-gradient GEMM X^T . Y from row-major operands (transposed ds_read_b64_tr_b16
    fragments of XOR-swizzled [64][128] images), split over rows into fp32 partials; at
    (256, 4096, 3136) the persistent kernel walks 400 tiles on 256 CUs."""
    from relayrl_prototype_amd.ops import hip

    monkeypatch.setenv("RRL_FC_BIG", big)
    h = hip()
    g = torch.Generator().manual_seed(R + I + J)
    x = _bf(torch.randn(R, I, generator=g))
    y = _bf(F.relu(torch.randn(R, J, generator=g)))
    part = torch.full((splits * I * J,), float("nan"), device=cuda)
    used = h.fc_tn_part(x.to(cuda).bfloat16().reshape(-1), y.to(cuda).bfloat16().reshape(-1), part, R, I, J, splits)
    assert 1 <= used <= splits
    got = part[:used * I * J].view(used, I, J).sum(0).cpu()
    ref = x.double().t() @ y.double()
    assert torch.isfinite(got).all()
    assert ((got.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
    if J % 128:  # bias gradient through the ones column of the padded last tile
        ones = torch.ones(8, dtype=torch.bfloat16, device=cuda)
        bp = torch.full((splits * I,), float("nan"), device=cuda)
        part.fill_(float("nan"))
        used2 = h.fc_tn_part(x.to(cuda).bfloat16().reshape(-1), y.to(cuda).bfloat16().reshape(-1), part, R, I, J,
                             splits, ones=ones, bias_part=bp)
        assert used2 == used
        assert torch.equal(part[:used * I * J].view(used, I, J).sum(0).cpu(), got)  # weights unchanged
        bsum = bp[:used * I].view(used, I).sum(0).cpu().double()
        bref = x.double().sum(0)
        assert ((bsum - bref).abs().max() / bref.abs().max()).item() < 1e-5


def test_persistent_fc_kernels_in_the_full_update(cuda, monkeypatch):
    """The 8,192-env sizes take the persistent 256 x 128 fc kernels (forward at >= 4,096 rows,
    weight + bias gradient at >= 20,480 rows): 5 rollout forwards of 4,096 rows and the backward
    over all 20,480 rows give the same gradient as the 128 x 128 kernels (RRL_FC_BIG=0) up to
    fp32 summation order and the bf16 rounding of the stored hidden units."""
    spec = CNNSpec(6)
    params = spec.init(11)
    N, T = 4096, 5
    B = N * T
    g = torch.Generator().manual_seed(2)
    obs = torch.randint(0, 256, (B, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    act = torch.randint(0, 6, (B,), dtype=torch.int32, generator=g).to(cuda)
    adv = torch.randn(B, generator=g).to(cuda)
    ret = torch.randn(B, generator=g).to(cuda)
    grads, hids = [], []
    for big in ("0", "1"):
        monkeypatch.setenv("RRL_FC_BIG", big)
        m = DeviceNatureCNN(spec, cuda, max_batch=B, params=params)
        a_out = torch.empty(N, dtype=torch.int32, device=cuda)
        lp, v = torch.empty(N, device=cuda), torch.empty(N, device=cuda)
        for t in range(T):
            m.act(obs[t * N:(t + 1) * N], t * N, a_out, lp, v, seed=1, step=t)
        m.backward(obs, act, adv, ret, 0.5, 0.01)
        torch.cuda.synchronize()
        grads.append(m.grad.clone())
        hids.append(m.hid[:B * HIDDEN].float().clone())
    assert torch.isfinite(grads[1]).all()
    assert relerr(hids[1], hids[0]) < 5e-3
    assert relerr(grads[1], grads[0]) < 1e-2


def test_sum_splits_multi_matches_torch(cuda):
    """Several slab sums in one launch (the conv layers' weight / bias partials)."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    g = torch.Generator(device=cuda).manual_seed(0)
    shapes = [(256, 36864), (2048, 64), (256, 32768), (7, 32), (1, 8)]
    segs, refs = [], []
    for s, n in shapes:
        p = torch.randn(s * n, device=cuda, generator=g)
        out = torch.full((n,), float("nan"), device=cuda)
        segs.append((p, s, n, out))
        refs.append(p.view(s, n).double().sum(0))
    h.sum_splits_multi(segs)
    for (_, s, n, out), ref in zip(segs, refs):
        assert torch.allclose(out.double(), ref, atol=1e-4, rtol=1e-5), (s, n)


@pytest.mark.parametrize("shapes", [[(5, 1605632), (5, 512)], [(1, 1028), (8, 64), (3, 4)]])
def test_sum_splits_few_matches_torch(cuda, shapes):
    """Few-split sums (every segment <= 8 splits: the fc weight / bias gradient's 5) take the
    one-column-per-thread launch."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    g = torch.Generator(device=cuda).manual_seed(1)
    segs, refs = [], []
    for s, n in shapes:
        p = torch.randn(s * n, device=cuda, generator=g)
        out = torch.full((n,), float("nan"), device=cuda)
        segs.append((p, s, n, out))
        refs.append(p.view(s, n).double().sum(0))
    h.sum_splits_multi(segs)
    for (_, s, n, out), ref in zip(segs, refs):
        assert torch.allclose(out.double(), ref, atol=1e-5, rtol=1e-6), (s, n)


def test_pong_step_render_fused_matches_separate(cuda):
    """One-launch step + render (a workgroup per env) == step kernel then render kernel, bitwise."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    N, S = 300, int(hip().pong_state_size())
    g = torch.Generator().manual_seed(3)
    st0 = torch.zeros(N * S, device=cuda)
    o1 = torch.empty(N, 21, 21, 64, dtype=torch.uint8, device=cuda)
    o2 = torch.empty_like(o1)
    z = [torch.zeros(N, device=cuda) for _ in range(4)]
    dummy = torch.zeros(N, dtype=torch.int32, device=cuda)
    h.pong_step(st0, dummy, *z, None, N, 11, 0, 400, True)
    s1, s2 = st0.clone(), st0.clone()
    acc1, acc2 = torch.zeros(4 * N, device=cuda), torch.zeros(4 * N, device=cuda)
    for t in range(1, 60):
        a = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
        r1 = [torch.zeros(N, device=cuda) for _ in range(4)]
        r2 = [torch.zeros(N, device=cuda) for _ in range(4)]
        h.pong_step(s1, a, *r1, acc1, N, 11, t, 400, False)
        h.pong_render(s1, o1, N)
        h.pong_step(s2, a, *r2, acc2, N, 11, t, 400, False, obs=o2)
        assert torch.equal(s1, s2) and torch.equal(o1, o2)
        assert all(torch.equal(x, y) for x, y in zip(r1, r2))
    assert torch.equal(acc1, acc2)


def test_pixel_update_side_stream_is_race_free(cuda, monkeypatch):
    """The head / fc weight gradients on the side stream (fork / join inside the captured
    update) give bitwise the same training trajectory as the single-stream backward: the two
    streams touch disjoint buffers and the join orders them before the optimiser."""
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    cfg = dict(num_envs=64, rollout_len=4, seed=5)
    runs = []
    for side, mode, defer, csums in (("0", "early", "0", "1"), ("1", "early", "0", "1"), ("1", "late", "0", "1"),
                                     ("1", "sums", "0", "1"), ("1", "early", "1", "1"), ("1", "early", "0", "0"),
                                     ("1", "early_main", "0", "1"), ("1", "early_fc", "0", "1"),
                                     ("1", "c3", "0", "1")):
        monkeypatch.setenv("RRL_CNN_SIDE_FC_FIRST", "1" if mode == "early_fc" else "0")
        mode = "early_main" if mode == "early_fc" else mode
        monkeypatch.setenv("RRL_CNN_SIDE", side)
        monkeypatch.setenv("RRL_CNN_SIDE_MODE", mode)
        monkeypatch.setenv("RRL_CNN_DEFER_TRANSPOSE", defer)
        monkeypatch.setenv("RRL_CNN_SIDE_CONV_SUMS", csums)
        tr = PixelA2CTrainer(PixelA2CConfig(use_graphs=True, **cfg), device=cuda)
        assert (tr.model.side_stream is not None) == (side == "1") and tr.model.side_mode == mode
        for _ in range(5):  # eager warm-up, capture + replay, 3 replays
            tr.train_epoch()
        torch.cuda.synchronize()
        runs.append(tr)
    b = runs[0]
    assert b._graph is not None
    for a in runs[1:]:
        assert a._graph is not None
        assert torch.equal(a.act, b.act) and torch.equal(a.obs, b.obs)
        torch.testing.assert_close(a.model.params, b.model.params, rtol=0, atol=0)
        torch.testing.assert_close(a.model.grad, b.model.grad, rtol=0, atol=0)


def test_pixel_update_16wave_backward_and_chunks(cuda, monkeypatch):
    """The 16-wave conv2 / conv3 backward kernels (bitwise equal to the 8-wave ones) train the
    same trajectory bitwise; conv2_bwd + conv1_wgrad8 in two row chunks (RRL_CNN_BWD21_CHUNKS)
    change only the grouping of the weight-gradient slab sums (fp32 reassociation)."""
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    cfg = dict(num_envs=300, rollout_len=4, seed=9)
    runs = []
    for b2, b3, chunks in (("0", "0", "1"), ("3", "1", "1"), ("0", "0", "2")):
        monkeypatch.setenv("RRL_CNN_FWD_LAYOUT", "128")
        monkeypatch.setenv("RRL_CNN_BWD2_VARIANT", b2)
        monkeypatch.setenv("RRL_CNN_BWD3_VARIANT", b3)
        monkeypatch.setenv("RRL_CNN_BWD21_CHUNKS", chunks)
        tr = PixelA2CTrainer(PixelA2CConfig(use_graphs=True, **cfg), device=cuda)
        for _ in range(3 if chunks == "1" else 1):
            tr.train_epoch()
        torch.cuda.synchronize()
        runs.append(tr)
    base, w16, ch = runs
    assert torch.equal(w16.act, base.act)
    torch.testing.assert_close(w16.model.params, base.model.params, rtol=0, atol=0)
    # one update from the same state: gradients equal up to fp32 summation order
    monkeypatch.setenv("RRL_CNN_BWD21_CHUNKS", "1")
    ref = PixelA2CTrainer(PixelA2CConfig(use_graphs=True, **cfg), device=cuda)
    ref.train_epoch()
    torch.cuda.synchronize()
    torch.testing.assert_close(ch.model.grad, ref.model.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(ch.model.params, ref.model.params, rtol=1e-4, atol=1e-6)


def _pong_histories(cuda, N, steps=40, seed=3):
    """Frame histories of N PongSynth envs after ``steps`` random-action steps, and the s2d
    observations the env's own step + render kernel drew for the same states."""
    from relayrl_prototype_amd.envs.pong import DevicePong

    env = DevicePong(N, cuda, seed)
    obs = torch.zeros(N, 21, 21, 64, dtype=torch.uint8, device=cuda)
    hist = torch.zeros(N, 16, device=cuda)
    env.reset(obs)
    g = torch.Generator().manual_seed(seed)
    for _ in range(steps):
        a = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
        env.step(a, obs)
    # the history rows of the same states (pong state layout: P_HIST = 16 .. 31)
    hist.copy_(env.state.view(N, -1)[:, 16:32])
    return hist, obs


@pytest.mark.parametrize("N", [37, 2048])
@pytest.mark.parametrize("wlds", ["0", "1"])  # RRL_PONG_HEAD_WLDS: head weights through LDS
def test_fused_head_step_equals_head_then_step(cuda, N, wlds, monkeypatch):
    """pong_head_step_render_kernel (the policy head inside the env-step launch) vs the head
    launch (a2c_head from the fc split-K partials) followed by the step + render launch: the
    same actions, log-probs, values, stored hidden units, env state, rewards, dones and
    rendered observations -- bitwise -- over several steps from mid-episode states."""
    import copy

    from relayrl_prototype_amd.envs.pong import DevicePong

    monkeypatch.setenv("RRL_PONG_HEAD_WLDS", wlds)
    spec = CNNSpec(6)
    m = DeviceNatureCNN(spec, cuda, max_batch=N, seed=5)
    envs = [DevicePong(N, cuda, 11), DevicePong(N, cuda, 11)]
    obs = [torch.zeros(N, 21, 21, 64, dtype=torch.uint8, device=cuda) for _ in range(2)]
    for e, o in zip(envs, obs):
        e.reset(o)
    sample_t = torch.full((1,), 3, dtype=torch.int64, device=cuda)
    for t in range(6):
        outs = []
        for k in range(2):
            act = torch.full((N,), -1, dtype=torch.int32, device=cuda)
            logp = torch.full((N,), float("nan"), device=cuda)
            val = torch.full((N,), float("nan"), device=cuda)
            rew = torch.full((N,), float("nan"), device=cuda)
            done = torch.full((N,), float("nan"), device=cuda)
            nxt = torch.zeros_like(obs[k])
            if k == 0:
                m.act(obs[k], 0, act, logp, val, 123, t, step_base=sample_t)
                envs[k].step(act, nxt, rew, done, offset=t)
            else:
                part, used, hid = m.forward_fc_partials(obs[k], 0)
                fc_b, hp = m.head_params()
                envs[k].step_head(part, used, fc_b, hp, m.A, hid, act, logp, val, 123, t, sample_t, nxt, rew, done,
                                  offset=t)
            torch.cuda.synchronize()
            outs.append((act.clone(), logp.clone(), val.clone(), m.hid[:N * 512].clone(), rew.clone(), done.clone(),
                         envs[k].state.clone()))
            obs[k] = nxt
        for a, b in zip(*outs):
            assert torch.equal(a, b)
        assert torch.equal(obs[0], obs[1])


@pytest.mark.parametrize("N", [37, 5000])
def test_streamed_rollout_head_is_bitwise_equal(cuda, N, monkeypatch):
    """a2c_head_streamed_kernel (RRL_HEAD_STREAMED=1: weights read per row, 79 VGPRs) gives
    the register-resident head's actions, log-probs, values and stored hidden units bitwise;
    N = 5000 runs 2 rows per wave on part of the grid (grid cap 1024).  Its backward twin
    gives the same gradients, dh and loss stats."""
    spec = CNNSpec(6)
    m = DeviceNatureCNN(spec, cuda, max_batch=N, seed=5)
    g = torch.Generator().manual_seed(3)
    obs = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    sample_t = torch.full((1,), 7, dtype=torch.int64, device=cuda)
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("RRL_HEAD_STREAMED", flag)
        act = torch.full((N,), -1, dtype=torch.int32, device=cuda)
        logp = torch.full((N,), float("nan"), device=cuda)
        val = torch.full((N,), float("nan"), device=cuda)
        m.hid.zero_()
        m.act(obs, 0, act, logp, val, 123, 4, step_base=sample_t)
        torch.cuda.synchronize()
        outs.append((act.clone(), logp.clone(), val.clone(), m.hid[:N * 512].clone()))
    assert (outs[0][0] >= 0).all()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # the streamed head backward (a2c_head_train_streamed_kernel): same gradients and loss stats
    act = outs[0][0]
    adv = torch.randn(N, generator=g).to(cuda)
    ret = torch.randn(N, generator=g).to(cuda)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("RRL_HEAD_STREAMED", flag)
        m.forward(obs, 0)
        stats = m.backward(obs, act, adv, ret, 0.5, 0.01)
        torch.cuda.synchronize()
        res.append((m.grad.clone(), stats.clone(), m.dh[:N * 512].clone()))
    assert res[0][1][:, 3].sum().item() == N
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N", [37, 5000])
def test_mfma_head_backward_matches_register_kernel(cuda, N, monkeypatch):
    """a2c_head_train_mfma_kernel (RRL_HEAD_MFMA=1: fp32 MFMA, exact f32 products summed in
    another order) vs a2c_head_kernel<true>: dhead / loss stats to fp32 rounding, dh to one bf16
    ulp where a sum lands on a rounding boundary, and the resulting gradients."""
    spec = CNNSpec(6)
    params = spec.init(2)
    o = spec.offsets()
    params[o["wpi"]:o["bpi"]] *= 50.0
    m = DeviceNatureCNN(spec, cuda, max_batch=N, params=params)
    g = torch.Generator().manual_seed(9)
    obs = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    act = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
    adv = torch.randn(N, generator=g).to(cuda)
    ret = torch.randn(N, generator=g).to(cuda)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("RRL_HEAD_MFMA", flag)
        m.forward(obs, 0)
        m.dh.fill_(float("nan"))
        m.dhead.fill_(float("nan"))
        stats = m.backward(obs, act, adv, ret, 0.5, 0.01)
        torch.cuda.synchronize()
        res.append((m.grad.clone(), stats.sum(0).cpu(), m.dh[:N * 512].float().cpu(),
                    m.dhead[:N * 7].clone().cpu()))
    (g0, s0, dh0, dd0), (g1, s1, dh1, dd1) = res
    assert torch.isfinite(dh1).all() and torch.isfinite(dd1).all()
    assert s1[3].item() == N
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dd1, dd0, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(dh1, dh0, rtol=8e-3, atol=1e-9)
    assert (dh1 == dh0).float().mean().item() > 0.9
    assert relerr(g1, g0) < 1e-3


def test_fused_render_draws_the_env_observation(cuda):
    """pong_render_hist(frame histories) == the observation pong_step's render wrote, bitwise;
    the history-output step kernel writes the same rows as the state's history slice."""
    from relayrl_prototype_amd.envs.pong import DevicePong
    from relayrl_prototype_amd.ops import hip

    N = 777
    hist, obs = _pong_histories(cuda, N)
    drawn = torch.full_like(obs, 7)
    hip().pong_render_hist(hist, drawn, N)
    torch.cuda.synchronize()
    assert torch.equal(drawn, obs)
    # step with hist_out: same physics, rows equal to the state's history
    e1, e2 = DevicePong(N, cuda, 5), DevicePong(N, cuda, 5)
    o = torch.zeros(N, 21, 21, 64, dtype=torch.uint8, device=cuda)
    h = torch.zeros(N, 16, device=cuda)
    e1.reset(o)
    e2.reset(hist_out=h)
    g = torch.Generator().manual_seed(1)
    for _ in range(30):
        a = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
        e1.step(a, o)
        e2.step(a, None, hist_out=h)
        torch.cuda.synchronize()
        assert torch.equal(e1.state, e2.state) and torch.equal(e1.rew, e2.rew) and torch.equal(e1.done, e2.done)
        assert torch.equal(h, e2.state.view(N, -1)[:, 16:32])
        hip().pong_render_hist(h, drawn[:N], N)
        assert torch.equal(drawn[:N], o)


@pytest.mark.parametrize("N", [5, 300, 2048])
def test_fused_render_conv_stack_equals_the_obs_path(cuda, N):
    """The 16-wave conv stack drawing its frames from histories (fused render) writes a1 / a2 / a3
    bitwise equal to the same kernel reading the rendered observations."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    spec = CNNSpec()
    o = spec.offsets()
    params = spec.init(N).to(cuda)
    params += 0.01 * torch.randn(params.shape, generator=torch.Generator().manual_seed(N)).to(cuda)
    sh = params.bfloat16()
    hist, obs = _pong_histories(cuda, N, seed=N)
    W = [sh[o["w1"]:o["b1"]], params[o["b1"]:o["b1"] + 32], sh[o["w2"]:o["b2"]], params[o["b2"]:o["b2"] + 64],
         sh[o["w3"]:o["b3"]], params[o["b3"]:o["b3"] + 64]]
    outs = []
    for fused in (False, True):
        a1 = torch.full((N * 400 * 32,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a2 = torch.full((N * 81 * 64,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a3 = torch.full((N * FC_IN,), float("nan"), dtype=torch.bfloat16, device=cuda)
        if fused:
            h.conv_stack_fwd(None, *W, a1, a2, a3, N, hist=hist)
        else:
            h.conv_stack_fwd(obs, *W, a1, a2, a3, N, probe=64)
        torch.cuda.synchronize()
        outs.append((a1, a2, a3))
    for f, r in zip(*outs):
        assert torch.isfinite(f.float()).all() and torch.equal(f, r)


def test_fused_render_conv1_wgrad_equals_the_obs_path(cuda):
    """conv1_wgrad8 drawing its frames from histories: weight and bias partials bitwise equal."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    N, grid = 1500, 256
    hist, obs = _pong_histories(cuda, N, seed=11)
    dy = torch.randn(N * 400 * 32, generator=torch.Generator().manual_seed(2)).bfloat16().to(cuda)
    outs = []
    for fused in (False, True):
        part = torch.full((2 * grid * 32 * 256,), float("nan"), device=cuda)
        bpart = torch.full((2 * grid * 32,), float("nan"), device=cuda)
        ns = h.conv1_wgrad8(None, dy, part, bpart, N, grid, hist=hist) if fused else \
            h.conv1_wgrad8(obs, dy, part, bpart, N, grid)
        torch.cuda.synchronize()
        outs.append((part[:ns * 32 * 256], bpart[:ns * 32]))
    for f, r in zip(*outs):
        assert torch.isfinite(f).all() and torch.equal(f, r)


def test_pixel_update_fused_render_matches_the_obs_path(cuda, monkeypatch):
    """A2C with the fused render (frame histories, no observation tensor) trains the same
    trajectory bitwise as with rendered observations (both on the 16-wave forward), captured."""
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    monkeypatch.setenv("RRL_CNN_FWD_LAYOUT", "64")
    runs = []
    for fused in (False, True):
        tr = PixelA2CTrainer(PixelA2CConfig(num_envs=300, rollout_len=4, seed=6, use_graphs=True,
                                            fused_render=fused, frame_ring=False), device=cuda)
        assert tr.fused_render == fused and tr.obs.dtype == (torch.float32 if fused else torch.uint8)
        for _ in range(5):
            tr.train_epoch()
        torch.cuda.synchronize()
        runs.append(tr)
    a, b = runs
    assert torch.equal(a.act, b.act) and torch.equal(a.rew, b.rew)
    torch.testing.assert_close(a.model.params, b.model.params, rtol=0, atol=0)
    assert a.metrics()["EnvSteps"] == b.metrics()["EnvSteps"]


def test_pixel_alternating_obs_buffers_match_copy_path(cuda, monkeypatch):
    """Two observation buffers used alternately (the last render of update k lands in slot 0 of
    update k + 1's buffer) train exactly like the single buffer + obs[T] -> obs[0] copy."""
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    cfg = dict(num_envs=64, rollout_len=4, seed=8)
    runs = []
    for copy in ("0", "1"):
        monkeypatch.setenv("RRL_PONG_OBS_COPY", copy)
        tr = PixelA2CTrainer(PixelA2CConfig(use_graphs=True, **cfg), device=cuda)
        assert len(tr._obs_bufs) == (1 if copy == "1" else 2)
        for _ in range(5):
            tr.train_epoch()
        torch.cuda.synchronize()
        runs.append(tr)
    a, b = runs
    assert torch.equal(a.obs[0], b.obs[0]) and torch.equal(a.act, b.act)  # the next update's start
    torch.testing.assert_close(a.model.params, b.model.params, rtol=0, atol=0)
    assert a.metrics()["EnvSteps"] == b.metrics()["EnvSteps"]


@pytest.mark.parametrize("base,probe", [(128, 16), (128, 32), (128, 48), (64, 80), (64, 96), (64, 112), (64, 68),
                                       (64, 65), (64, 72), (64, 73)])
def test_fused_conv_stack_layout_variants_are_bitwise_equal(cuda, base, probe):
    """The forward's LDS layout variants (FwdLayout probe bits: a1 as stride-2 phase images with
    conv2 over a 9 x 10 grid, conv3 over a 7 x 9 grid) run the same MFMA k-order per output:
    a1 / a2 / a3 bitwise equal to the default layout's, discarded grid positions never stored."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    spec = CNNSpec()
    o = spec.offsets()
    N = 700
    g = torch.Generator().manual_seed(probe)
    params = spec.init(probe).to(cuda)
    params += 0.01 * torch.randn(params.shape, generator=g).to(cuda)
    sh = params.bfloat16()
    x = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    outs = []
    for pr in (base, probe):  # base 128: the 8-wave kernel, 64: the 16-wave kernel (+ layout bits)
        a1 = torch.full((N * 400 * 32,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a2 = torch.full((N * 81 * 64,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a3 = torch.full((N * FC_IN,), float("nan"), dtype=torch.bfloat16, device=cuda)
        h.conv_stack_fwd(x, sh[o["w1"]:o["b1"]], params[o["b1"]:o["b1"] + 32], sh[o["w2"]:o["b2"]],
                         params[o["b2"]:o["b2"] + 64], sh[o["w3"]:o["b3"]], params[o["b3"]:o["b3"] + 64], a1, a2, a3,
                         N, probe=pr)
        torch.cuda.synchronize()
        outs.append((a1, a2, a3))
    for f, r in zip(*outs):
        assert torch.isfinite(f.float()).all()
        assert torch.equal(f, r)


@pytest.mark.parametrize("variant", [128, 64], ids=["8wave", "16wave"])
def test_fused_conv_stack_without_stored_activations(cuda, variant):
    """The bootstrap forward (no backward reads a1 / a2: y1 / y2 not written) leaves a3 bitwise
    equal to the full forward's and the a1 / a2 buffers untouched -- both kernels, with frames
    that do not divide the grid (workgroups with 2 and 3 frames, the pipeline drain)."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    spec = CNNSpec()
    o = spec.offsets()
    N = 700
    g = torch.Generator().manual_seed(variant)
    params = spec.init(variant).to(cuda)
    params += 0.01 * torch.randn(params.shape, generator=g).to(cuda)
    sh = params.bfloat16()
    x = torch.randint(0, 256, (N, 21, 21, 64), dtype=torch.uint8, generator=g).to(cuda)
    outs = []
    for store12 in (True, False):
        a1 = torch.full((N * 400 * 32,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a2 = torch.full((N * 81 * 64,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a3 = torch.full((N * FC_IN,), float("nan"), dtype=torch.bfloat16, device=cuda)
        h.conv_stack_fwd(x, sh[o["w1"]:o["b1"]], params[o["b1"]:o["b1"] + 32], sh[o["w2"]:o["b2"]],
                         params[o["b2"]:o["b2"] + 64], sh[o["w3"]:o["b3"]], params[o["b3"]:o["b3"] + 64], a1, a2, a3,
                         N, probe=variant, store12=store12)
        torch.cuda.synchronize()
        outs.append((a1, a2, a3))
    assert torch.isfinite(outs[0][2].float()).all()
    assert torch.equal(outs[0][2], outs[1][2])
    assert torch.isnan(outs[1][0].float()).all() and torch.isnan(outs[1][1].float()).all()


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6],
                         ids=["16wave", "no_setprio", "setprio_static", "setprio_wgrad", "setprio_dgrad", "16wave_setprio"])
def test_conv3_bwd_16wave_is_bitwise_equal(cuda, variant):
    """The 16-wave conv3 backward (dgrad and wgrad on separate waves) runs the 8-wave kernel's
    k-order per output: da2, the weight and the bias partials bitwise equal; so do the other
    wave-priority forms (2: none, 3: static) of the 8-wave kernel (shipped: s_setprio clusters)."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    L = CONVS[2]
    N, grid = 333, 64
    g = torch.Generator().manual_seed(13)
    x = torch.relu(torch.randn(N * L.hin * L.hin * L.cin, generator=g)).bfloat16().to(cuda)
    w = (torch.randn(L.cout * L.K, generator=g) * 0.05).bfloat16().to(cuda)
    dy = torch.randn(N * L.hout * L.hout * L.cout, generator=g).bfloat16().to(cuda)
    outs = []
    for v in (0, variant):
        dx = torch.full((N * L.hin * L.hin * L.cin,), float("nan"), dtype=torch.bfloat16, device=cuda)
        part = torch.full((grid * L.cout * L.K,), float("nan"), device=cuda)
        bpart = torch.full((grid * 512,), float("nan"), device=cuda)
        h.conv3_bwd(dy, w, x, dx, part, bpart, N, grid, variant=v)
        torch.cuda.synchronize()
        outs.append((dx, part, bpart[:grid * 64]))
    for a, b in zip(*outs):
        assert torch.isfinite(a.float()).all() and torch.equal(a, b)


@pytest.mark.parametrize("variant", [2, 3, 4, 5, 6, 7, 8],
                         ids=["grid12", "16wave", "setprio", "setprio_static", "setprio_wgrad", "setprio_dgrad",
                              "store16"])
def test_conv2_bwd_dgrad_grids_are_bitwise_equal(cuda, variant):
    """The conv2 backward's dgrad over the class's 100 pixels in 7 tiles (shipped) against the
    dgrad over a 10 x 12 grid per phase class (variant 2) and the 16-wave kernel with dgrad and
    wgrad on separate waves (variant 3): the same k-order per output, so da1, the weight and the
    bias partials are bitwise equal."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    L = CONVS[1]
    N, grid = 333, 64
    g = torch.Generator().manual_seed(12)
    x = torch.relu(torch.randn(N * L.hin * L.hin * L.cin, generator=g)).bfloat16().to(cuda)
    w = (torch.randn(L.cout * L.K, generator=g) * 0.05).bfloat16().to(cuda)
    dy = torch.randn(N * L.hout * L.hout * L.cout, generator=g).bfloat16().to(cuda)
    outs = []
    for v in (0, variant):
        dx = torch.full((N * L.hin * L.hin * L.cin,), float("nan"), dtype=torch.bfloat16, device=cuda)
        part = torch.full((grid * L.cout * L.K,), float("nan"), device=cuda)
        bpart = torch.full((grid * 512,), float("nan"), device=cuda)
        h.conv2_bwd(dy, w, x, dx, part, bpart, N, grid, staged=v)
        torch.cuda.synchronize()
        outs.append((dx, part, bpart[:grid * 64]))  # one 64-channel bias partial per workgroup
    for a, b in zip(*outs):
        assert torch.isfinite(a.float()).all() and torch.equal(a, b)
