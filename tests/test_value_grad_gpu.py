"""The weight-stationary bf16x6 value-gradient kernel (csrc/kernels/value_grad.hip).

It replaces the fp32-MFMA kernel for the value step (train_vf_iters = 80 per epoch,
REINFORCE.py:110-115) when H = 128 and D <= 24.  Its products run on bf16 matrix cores with
every fp32 operand split three ways, so it must be as accurate as fp32 math: both kernels
are compared against a float64 autograd oracle of the same loss, and the split kernel's
error may not exceed the fp32 kernel's by more than a small factor.
"""
import pytest
import torch

from relayrl_prototype_amd.ops import GradHead, MLPSpec, mlp_grad, set_value_grad_mode

pytestmark = pytest.mark.gpu


def _grad64(params, X, ret, D, H, inv_B):
    p = params.double().clone().requires_grad_(True)
    o = 0
    W1 = p[o:o + H * D].view(H, D); o += H * D
    b1 = p[o:o + H]; o += H
    W2 = p[o:o + H * H].view(H, H); o += H * H
    b2 = p[o:o + H]; o += H
    W3 = p[o:o + H].view(1, H); o += H
    b3 = p[o:o + 1]
    h1 = torch.relu(X.double() @ W1.T + b1)
    h2 = torch.relu(h1 @ W2.T + b2)
    v = (h2 @ W3.T + b3)[:, 0]
    loss = ((v - ret.double()) ** 2).sum() * inv_B
    loss.backward()
    return p.grad, ((v - ret.double()) ** 2).sum().item()


def _away_from_relu_kinks(params, X, D, H, tau=1e-5):
    """Rows whose hidden pre-activations are all at least tau away from 0 in float64.

    Any two fp32-accurate evaluations of the same net differ by ~1e-7 in a pre-activation,
    so where one lies within that of the ReLU kink the two can take opposite sides of it and
    their gradients then legitimately differ by a whole row's contribution.  Dropping the
    ~0.1 % of rows with a pre-activation inside +-1e-5 makes the comparison a test of the
    arithmetic only."""
    p = params.double()
    o = 0
    W1 = p[o:o + H * D].view(H, D); o += H * D
    b1 = p[o:o + H]; o += H
    W2 = p[o:o + H * H].view(H, H); o += H * H
    b2 = p[o:o + H]
    z1 = X.double() @ W1.T + b1
    z2 = torch.relu(z1) @ W2.T + b2
    m = torch.minimum(z1.abs().min(1).values, z2.abs().min(1).values)
    return m > tau


def _run(mode, pp, X, ret, H):
    old = set_value_grad_mode(mode)
    try:
        slab, loss = mlp_grad(GradHead.VALUE_MSE, pp, X, 1, H, ret=ret)
        torch.cuda.synchronize()
    finally:
        set_value_grad_mode(old)
    return slab.sum(0, dtype=torch.float64).cpu(), loss.sum(0).cpu()


@pytest.mark.parametrize("D,B", [(4, 1), (4, 63), (4, 5000), (4, 70000), (8, 33000), (2, 777), (6, 4097), (3, 16),
                                 (11, 3000), (16, 4100), (17, 33000), (19, 5000), (20, 3000), (24, 777)])
def test_split_kernel_matches_float64(cuda, D, B):
    H = 128
    g = torch.Generator().manual_seed(D * 1000 + B)
    spec = MLPSpec(D, H, 1, False)
    pp = spec.init(g)
    pp = pp + 0.05 * torch.randn(pp.shape, generator=g)  # non-zero biases, generic weights
    X = torch.randn(B, D, generator=g) * 1.5
    ret = torch.randn(B, generator=g) * 20 + 5
    keep = _away_from_relu_kinks(pp, X, D, H)
    X, ret = X[keep], ret[keep]
    B = X.shape[0]
    g64, loss64 = _grad64(pp, X, ret, D, H, 1.0 / B)
    gs, ls = _run(1, pp.to(cuda), X.to(cuda), ret.to(cuda), H)
    gf, lf = _run(0, pp.to(cuda), X.to(cuda), ret.to(cuda), H)
    scale = g64.abs().max().item()
    err_split = (gs - g64).abs().max().item() / scale
    err_fp32 = (gf - g64).abs().max().item() / scale
    # fp32-level: both within a few fp32 ulps of the largest gradient entry, and the split
    # kernel no worse than twice the fp32 kernel's error
    assert err_fp32 < 1e-5, err_fp32
    assert err_split < 1e-5, (err_split, err_fp32)
    assert err_split <= 2.0 * err_fp32 + 2e-7, (err_split, err_fp32)
    assert abs(ls[0].item() - loss64) <= 1e-5 * abs(loss64) + 1e-6
    assert int(ls[5].item()) == B
    assert ls[1:4].abs().sum().item() == 0.0


@pytest.mark.parametrize("tune", [128, 144, 176])  # V = 0 (hi-piece dh1), 1 (mask table), 3 (+ interleaved)
@pytest.mark.parametrize("B", [5000, 70000])
@pytest.mark.parametrize("D", [4, 8])
def test_split_kernel_variants_match_float64(cuda, tune, B, D):
    """Every structural variant of the factored value head (value_grad.hip vg_prod_v) is as
    accurate as the fp32 kernel and bitwise deterministic."""
    from relayrl_prototype_amd.ops import hip

    H = 128
    g = torch.Generator().manual_seed(B + tune + D)
    pp = MLPSpec(D, H, 1, False).init(g)
    pp = pp + 0.05 * torch.randn(pp.shape, generator=g)
    X = torch.randn(B, D, generator=g) * 1.5
    ret = torch.randn(B, generator=g) * 20 + 5
    keep = _away_from_relu_kinks(pp, X, D, H)
    X, ret = X[keep], ret[keep]
    B = X.shape[0]
    g64, loss64 = _grad64(pp, X, ret, D, H, 1.0 / B)
    old = hip().set_value_grad_tune(tune)
    try:
        gs, ls = _run(1, pp.to(cuda), X.to(cuda), ret.to(cuda), H)
        gs2, _ = _run(1, pp.to(cuda), X.to(cuda), ret.to(cuda), H)
    finally:
        hip().set_value_grad_tune(old)
    gf, _ = _run(0, pp.to(cuda), X.to(cuda), ret.to(cuda), H)
    scale = g64.abs().max().item()
    err_split = (gs - g64).abs().max().item() / scale
    err_fp32 = (gf - g64).abs().max().item() / scale
    assert err_split < 1e-5 and err_split <= 2.0 * err_fp32 + 2e-7, (err_split, err_fp32)
    assert abs(ls[0].item() - loss64) <= 1e-5 * abs(loss64) + 1e-6
    assert torch.equal(gs, gs2)


def test_mode_switch_roundtrip(cuda):
    old = set_value_grad_mode(-1)
    assert old in (0, 1)
    assert set_value_grad_mode(0) == old
    assert set_value_grad_mode(-1) == 0
    assert set_value_grad_mode(old) == 0
    assert set_value_grad_mode(-1) == old


@pytest.mark.parametrize("D,B", [(4, 32768), (2, 20000), (8, 33000), (17, 20000)])
def test_deterministic(cuda, D, B):
    """Bitwise identical partial-gradient slabs across repeated launches (the slabs are
    reduced in a fixed order by adam.hip, so the whole update is reproducible)."""
    H = 128
    g = torch.Generator().manual_seed(7 * D + B)
    spec = MLPSpec(D, H, 1, False)
    pp = (spec.init(g) + 0.05 * torch.randn(spec.P, generator=g)).to(cuda)
    X = (torch.randn(B, D, generator=g) * 1.5).to(cuda)
    ret = (torch.randn(B, generator=g) * 20 + 5).to(cuda)
    old = set_value_grad_mode(1)
    try:
        ref, _ = mlp_grad(GradHead.VALUE_MSE, pp, X, 1, H, ret=ret)
        ref = ref.clone()
        for _ in range(12):
            s, _ = mlp_grad(GradHead.VALUE_MSE, pp, X, 1, H, ret=ret)
            assert torch.equal(s, ref)
    finally:
        set_value_grad_mode(old)


@pytest.mark.parametrize("D,B,shift", [(4, 20000, 1), (4, 20000, 2), (8, 9000, 3), (17, 9000, 1)])
def test_unaligned_params_slice(cuda, D, B, shift):
    """The prologue stages W2 with 16-byte loads when the params slice allows and with element
    loads otherwise: a params view at a 4-byte (not 16-byte) offset gives bitwise the same slabs."""
    H = 128
    g = torch.Generator().manual_seed(11 * D + shift)
    spec = MLPSpec(D, H, 1, False)
    pp = (spec.init(g) + 0.05 * torch.randn(spec.P, generator=g)).to(cuda)
    buf = torch.zeros(spec.P + 8, device=cuda)
    buf[shift:shift + spec.P] = pp
    pv = buf[shift:shift + spec.P]
    assert pv.data_ptr() % 16 != 0
    X = (torch.randn(B, D, generator=g) * 1.5).to(cuda)
    ret = (torch.randn(B, generator=g) * 20 + 5).to(cuda)
    old = set_value_grad_mode(1)
    try:
        ref, lref = mlp_grad(GradHead.VALUE_MSE, pp, X, 1, H, ret=ret)
        ref, lref = ref.clone(), lref.clone()
        s, ls = mlp_grad(GradHead.VALUE_MSE, pv, X, 1, H, ret=ret)
        assert torch.equal(s, ref)
        assert torch.equal(ls, lref)
    finally:
        set_value_grad_mode(old)


def _pg64(head, pp, X, A, H, mask, act, adv, logp_old, stats, inv_B, clip, ent_coef):
    """float64 autograd gradient of the categorical PG / PPO loss (mlp_grad.hip semantics:
    normalised advantages, masked logits, entropy bonus, true log_softmax log-probs)."""
    D = X.shape[1]
    p = pp.double().clone().requires_grad_(True)
    o = 0
    W1 = p[o:o + H * D].view(H, D); o += H * D
    b1 = p[o:o + H]; o += H
    W2 = p[o:o + H * H].view(H, H); o += H * H
    b2 = p[o:o + H]; o += H
    W3 = p[o:o + A * H].view(A, H); o += A * H
    b3 = p[o:o + A]
    h = torch.relu(torch.relu(X.double() @ W1.T + b1) @ W2.T + b2)
    lsm = torch.log_softmax(h @ W3.T + b3 + (mask.double() - 1.0) * 1e8, -1)
    logp = lsm.gather(1, act.long()[:, None])[:, 0]
    n = float(stats[2])
    mean = float(stats[0]) / n
    var = max(float(stats[1]) / n - mean * mean, 0.0)
    advn = (adv.double() - mean) / (var ** 0.5 + 1e-8)
    if head == "PG_CAT":
        li = -logp * advn
    else:
        ratio = torch.exp(logp - logp_old.double())
        li = -torch.minimum(ratio * advn, torch.clamp(ratio, 1 - clip, 1 + clip) * advn)
    ent = -(lsm.exp() * lsm).sum(-1)
    ((li.sum() - ent_coef * ent.sum()) * inv_B).backward()
    return p.grad.detach()


@pytest.mark.parametrize("head", ["PG_CAT", "PPO_CAT"])
@pytest.mark.parametrize("D,B,A", [(4, 5000, 2), (4, 70000, 2), (3, 777, 2), (8, 33000, 2), (2, 4097, 3),
                                   (6, 20000, 3), (8, 33000, 4), (4, 999, 4)])
def test_policy_split_kernel_matches_oracle(cuda, head, D, B, A):
    """Categorical policy heads (A = 2..4: CartPole, MountainCar / Acrobot, LunarLander) on the
    bf16x6 kernel against the fp32-MFMA kernel and the autograd oracle: masks, advantage
    normalisation, PPO ratio clipping, entropy bonus and the loss statistics."""
    H = 128
    hd = getattr(GradHead, head)
    g = torch.Generator().manual_seed(D * 31 + B)
    spec = MLPSpec(D, H, A, False)
    pp = spec.init(g)
    pp = pp + 0.05 * torch.randn(pp.shape, generator=g)
    X = torch.randn(B, D, generator=g) * 1.5
    keep = _away_from_relu_kinks(pp, X, D, H)
    X = X[keep]
    B = X.shape[0]
    act = torch.randint(0, A, (B,), generator=g, dtype=torch.int32)
    adv = torch.randn(B, generator=g) * 3 + 0.5
    mask = torch.ones(B, A)
    mask[torch.arange(B) % 97 == 5, A - 1] = 0.0
    act[torch.arange(B) % 97 == 5] = 0
    logp_old = -torch.rand(B, generator=g) * 1.2 - 0.05
    stats = torch.tensor([adv.sum().item(), (adv * adv).sum().item(), float(B)])
    kw = dict(mask=mask, act=act, adv=adv, logp_old=logp_old, adv_stats=stats, inv_B=1.0 / B, clip_eps=0.2,
              ent_coef=0.01)
    g_ref = _pg64(head, pp, X, A, H, mask, act, adv, logp_old, stats, 1.0 / B, 0.2, 0.01)
    out = {}
    for mode in (1, 0):
        old = set_value_grad_mode(mode)
        try:
            kwc = {k: (v.to(cuda) if torch.is_tensor(v) else v) for k, v in kw.items()}
            slab, loss = mlp_grad(hd, pp.to(cuda), X.to(cuda), A, H, **kwc)
            torch.cuda.synchronize()
        finally:
            set_value_grad_mode(old)
        out[mode] = (slab.sum(0, dtype=torch.float64).cpu(), loss.sum(0).cpu())
    scale = g_ref.abs().max().item()
    err_split = (out[1][0] - g_ref).abs().max().item() / scale
    err_fp32 = (out[0][0] - g_ref).abs().max().item() / scale
    assert err_fp32 < 1e-5, err_fp32
    assert err_split < 1e-5, (err_split, err_fp32)
    ls, lf = out[1][1], out[0][1]
    assert int(ls[5].item()) == B and int(lf[5].item()) == B
    for k, name in ((0, "loss"), (1, "entropy"), (2, "kl"), (3, "clipfrac")):
        assert abs(ls[k].item() - lf[k].item()) <= 1e-4 * max(1.0, abs(lf[k].item())), (name, ls[k], lf[k])


def _gauss64(head, pp, X, A, H, actc, adv, logp_old, stats, inv_B, clip, ent_coef):
    """float64 autograd gradient of the diagonal-Gaussian PG / PPO loss (mlp_grad.hip
    HEAD_PG_GAUSS / HEAD_PPO_GAUSS: state-independent log_std, entropy bonus)."""
    import math

    D = X.shape[1]
    p = pp.double().clone().requires_grad_(True)
    o = 0
    W1 = p[o:o + H * D].view(H, D); o += H * D
    b1 = p[o:o + H]; o += H
    W2 = p[o:o + H * H].view(H, H); o += H * H
    b2 = p[o:o + H]; o += H
    W3 = p[o:o + A * H].view(A, H); o += A * H
    b3 = p[o:o + A]; o += A
    ls = p[o:o + A]
    mu = torch.relu(torch.relu(X.double() @ W1.T + b1) @ W2.T + b2) @ W3.T + b3
    z = (actc.double() - mu) * torch.exp(-ls)
    logp = (-0.5 * z * z - ls - 0.5 * math.log(2 * math.pi)).sum(-1)
    n = float(stats[2])
    mean = float(stats[0]) / n
    var = max(float(stats[1]) / n - mean * mean, 0.0)
    advn = (adv.double() - mean) / (var ** 0.5 + 1e-8)
    if head == "PG_GAUSS":
        li = -logp * advn
    else:
        ratio = torch.exp(logp - logp_old.double())
        li = -torch.minimum(ratio * advn, torch.clamp(ratio, 1 - clip, 1 + clip) * advn)
    ent = (0.5 + 0.5 * math.log(2 * math.pi) + ls).sum() * X.shape[0]
    ((li.sum() - ent_coef * ent) * inv_B).backward()
    return p.grad.detach(), logp.detach()


@pytest.mark.parametrize("head", ["PG_GAUSS", "PPO_GAUSS"])
@pytest.mark.parametrize("D,B,A", [(17, 33000, 6), (17, 777, 6), (20, 5000, 6), (3, 20000, 1), (8, 4097, 6)])
def test_gaussian_split_kernel_matches_oracle(cuda, head, D, B, A):
    """Diagonal-Gaussian policy heads (HalfCheetah A = 6, Pendulum A = 1) on the bf16x6 kernel
    against the float64 oracle and the fp32-MFMA kernel, including the log_std gradient."""
    H = 128
    hd = getattr(GradHead, head)
    g = torch.Generator().manual_seed(D * 17 + B + A)
    spec = MLPSpec(D, H, A, True)
    pp = spec.init(g, log_std_init=-0.5)
    pp = pp + 0.05 * torch.randn(pp.shape, generator=g)
    X = torch.randn(B, D, generator=g) * 1.5
    keep = _away_from_relu_kinks(pp, X, D, H)
    X = X[keep]
    B = X.shape[0]
    actc = torch.randn(B, A, generator=g) * 0.7
    adv = torch.randn(B, generator=g) * 3 + 0.5
    stats = torch.tensor([adv.sum().item(), (adv * adv).sum().item(), float(B)])
    _, logp_now = _gauss64("PG_GAUSS", pp, X, A, H, actc, adv, None, stats, 1.0 / B, 0.2, 0.01)
    logp_old = (logp_now + 0.3 * torch.randn(B, generator=g, dtype=torch.float64)).float()
    # the clipped surrogate is discontinuous at ratio = 1 +- clip: rows whose float64 ratio lies
    # within 1e-4 of it can fall on either side for any two fp32-accurate evaluations (and one
    # such row moves a gradient entry by ~1e-4 of its scale), so they are left out, like the
    # ReLU kinks above
    ratio = torch.exp(logp_now - logp_old.double())
    far = ((ratio - 1.2).abs() > 1e-4) & ((ratio - 0.8).abs() > 1e-4)
    X, actc, adv, logp_old = X[far], actc[far], adv[far], logp_old[far]
    B = X.shape[0]
    stats = torch.tensor([adv.sum().item(), (adv * adv).sum().item(), float(B)])
    kw = dict(actc=actc, adv=adv, logp_old=logp_old, adv_stats=stats, inv_B=1.0 / B, clip_eps=0.2, ent_coef=0.01)
    g_ref, _ = _gauss64(head, pp, X, A, H, actc, adv, logp_old, stats, 1.0 / B, 0.2, 0.01)
    out = {}
    for mode in (1, 0):
        old = set_value_grad_mode(mode)
        try:
            kwc = {k: (v.to(cuda) if torch.is_tensor(v) else v) for k, v in kw.items()}
            slab, loss = mlp_grad(hd, pp.to(cuda), X.to(cuda), A, H, **kwc)
            torch.cuda.synchronize()
        finally:
            set_value_grad_mode(old)
        out[mode] = (slab.sum(0, dtype=torch.float64).cpu(), loss.sum(0).cpu())
    scale = g_ref.abs().max().item()
    err_split = (out[1][0] - g_ref).abs().max().item() / scale
    err_fp32 = (out[0][0] - g_ref).abs().max().item() / scale
    assert err_fp32 < 1e-5, err_fp32
    assert err_split < 1e-5, (err_split, err_fp32)
    ls, lf = out[1][1], out[0][1]
    assert int(ls[5].item()) == B and int(lf[5].item()) == B
    for k, name in ((0, "loss"), (1, "entropy"), (2, "kl"), (3, "clipfrac")):
        assert abs(ls[k].item() - lf[k].item()) <= 1e-4 * max(1.0, abs(lf[k].item())), (name, ls[k], lf[k])


def _v64(params, X, D, H):
    p = params.double()
    o = 0
    W1 = p[o:o + H * D].view(H, D); o += H * D
    b1 = p[o:o + H]; o += H
    W2 = p[o:o + H * H].view(H, H); o += H * H
    b2 = p[o:o + H]; o += H
    W3 = p[o:o + H].view(1, H); o += H
    b3 = p[o:o + 1]
    return (torch.relu(torch.relu(X.double() @ W1.T + b1) @ W2.T + b2) @ W3.T + b3)[:, 0]


@pytest.mark.parametrize("D,B", [(4, 1), (4, 63), (4, 70001), (8, 33000), (3, 777), (17, 20000), (24, 4097)])
def test_value_forward_split_matches_float64(cuda, D, B):
    """The value forward on the bf16x6 weight-stationary kernel (value_grad.hip FWD instance)
    is fp32-accurate: against float64 no worse than twice the fp32-MFMA forward's error."""
    from relayrl_prototype_amd.ops import FwdMode, hip, mlp_forward

    H = 128
    g = torch.Generator().manual_seed(D * 7 + B)
    pp = MLPSpec(D, H, 1, False).init(g)
    pp = pp + 0.05 * torch.randn(pp.shape, generator=g)
    X = torch.randn(B, D, generator=g) * 1.5
    v64 = _v64(pp, X, D, H)
    out = {}
    for mode in (1, 0):
        old = hip().set_value_fwd_mode(mode)
        try:
            out[mode] = mlp_forward(FwdMode.VALUE, pp.to(cuda), X.to(cuda), 1, H)["v"].double().cpu().reshape(-1)
        finally:
            hip().set_value_fwd_mode(old)
    scale = max(v64.abs().max().item(), 1e-3)
    err_split = (out[1] - v64).abs().max().item() / scale
    err_fp32 = (out[0] - v64).abs().max().item() / scale
    assert err_fp32 < 1e-5, err_fp32
    assert err_split < 1e-5 and err_split <= 2.0 * err_fp32 + 2e-7, (err_split, err_fp32)


def test_value_forward_mode_switch(cuda):
    from relayrl_prototype_amd.ops import hip

    old = hip().set_value_fwd_mode(-1)
    assert old in (0, 1)
    assert hip().set_value_fwd_mode(0) == old
    assert hip().set_value_fwd_mode(old) == 0


@pytest.mark.parametrize("head", ["VALUE_MSE", "PG_CAT", "PPO_CAT"])
@pytest.mark.parametrize("D,A", [(4, 2), (8, 4)])
def test_device_row_count_matches_a_cut_batch(cuda, head, D, A):
    """grad_args.h nvalid / inv_B_dev: a capacity batch whose rows >= nvalid hold garbage (NaN)
    gives the gradient of the first nvalid rows with the device inv_B (graph replays with a
    changing agent-row count, rollout_learn.py)."""
    H = 128
    hd = getattr(GradHead, head)
    Aeff = 1 if head == "VALUE_MSE" else A
    g = torch.Generator().manual_seed(D * 131 + A)
    pp = MLPSpec(D, H, Aeff, False).init(g)
    pp = (pp + 0.05 * torch.randn(pp.shape, generator=g)).to(cuda)
    cap, n = 9000, 5123
    X = torch.randn(cap, D, generator=g).to(cuda)
    X[n:] = float("nan")
    ret = (torch.randn(cap, generator=g) * 5).to(cuda)
    adv = torch.randn(cap, generator=g).to(cuda)
    act = torch.randint(0, A, (cap,), generator=g, dtype=torch.int32).to(cuda)
    lpo = (-torch.rand(cap, generator=g)).to(cuda)
    stats = torch.tensor([adv[:n].sum().item(), (adv[:n] ** 2).sum().item(), float(n)], device=cuda)
    kw = dict(ret=ret, adv=adv, act=act, logp_old=lpo, adv_stats=stats, mask=None, ent_coef=0.01)
    if head == "VALUE_MSE":
        kw = dict(ret=ret)
    nv = torch.tensor([n], dtype=torch.int32, device=cuda)
    ibd = torch.tensor([1.0 / 7777.0], device=cuda)
    old = set_value_grad_mode(1)
    try:
        s_dev, l_dev = mlp_grad(hd, pp, X, A, H, inv_B=0.5, nvalid=nv, inv_B_dev=ibd, **kw)
        s_dev = s_dev.sum(0, dtype=torch.float64)
        l_dev = l_dev.sum(0)
        cut = {k: (v[:n] if (torch.is_tensor(v) and k != "adv_stats") else v) for k, v in kw.items()}
        s_ref, l_ref = mlp_grad(hd, pp, X[:n], A, H, inv_B=1.0 / 7777.0, **cut)
        s_ref = s_ref.sum(0, dtype=torch.float64)
        l_ref = l_ref.sum(0)
        torch.cuda.synchronize()
    finally:
        set_value_grad_mode(old)
    assert torch.isfinite(s_dev).all()
    scale = s_ref.abs().max().item()
    assert (s_dev - s_ref).abs().max().item() <= 1e-6 * scale, (s_dev - s_ref).abs().max().item() / scale
    assert int(l_dev[5].item()) == n
    assert abs(l_dev[0].item() - l_ref[0].item()) <= 1e-5 * max(1.0, abs(l_ref[0].item()))


def test_binary_policy_head_factored_is_deterministic(cuda):
    """The 2-action categorical head on the rank-1 factored path (dlogit0 = -dlogit1) gives
    bitwise identical slabs across launches."""
    H, D, A, B = 128, 4, 2, 40000
    g = torch.Generator().manual_seed(99)
    pp = (MLPSpec(D, H, A, False).init(g) + 0.05 * torch.randn(MLPSpec(D, H, A, False).P, generator=g)).to(cuda)
    X = torch.randn(B, D, generator=g).to(cuda)
    act = torch.randint(0, A, (B,), generator=g, dtype=torch.int32).to(cuda)
    adv = torch.randn(B, generator=g).to(cuda)
    stats = torch.tensor([adv.sum().item(), (adv * adv).sum().item(), float(B)], device=cuda)
    old = set_value_grad_mode(1)
    try:
        ref, _ = mlp_grad(GradHead.PG_CAT, pp, X, A, H, act=act, adv=adv, adv_stats=stats)
        ref = ref.clone()
        for _ in range(5):
            s, _ = mlp_grad(GradHead.PG_CAT, pp, X, A, H, act=act, adv=adv, adv_stats=stats)
            assert torch.equal(s, ref)
    finally:
        set_value_grad_mode(old)
