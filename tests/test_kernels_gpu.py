"""Numerics of every HIP kernel against the PyTorch fp32 oracle (ops/reference.py)."""
import numpy as np
import pytest
import torch

from relayrl_prototype_amd.ops import FwdMode, GradHead, MLPSpec, mlp_forward, mlp_grad, gae_scan_tm, scan_flat
from relayrl_prototype_amd.ops import adam_step, reduce_slabs
from relayrl_prototype_amd.ops import reference as ref
from relayrl_prototype_amd.ops import philox

pytestmark = pytest.mark.gpu

SHAPES = [(4, 128, 2, 1), (4, 128, 2, 1000), (8, 128, 4, 257), (2, 64, 3, 100), (17, 128, 6, 333), (6, 64, 3, 16)]


def _params(spec, seed=0):
    g = torch.Generator().manual_seed(seed)
    return spec.init(g)


@pytest.mark.parametrize("D,H,A,B", SHAPES)
def test_forward_value_logits_eval(cuda, D, H, A, B):
    torch.manual_seed(D * 1000 + B)
    X = torch.randn(B, D)
    mask = (torch.rand(B, A) > 0.2).float()
    mask[:, 0] = 1.0
    act = torch.randint(0, A, (B,), dtype=torch.int32)
    act = torch.where(mask.gather(1, act.long().unsqueeze(1)).squeeze(1) > 0, act, torch.zeros_like(act))
    pv = _params(MLPSpec(D, H, 1), 1)
    pp = _params(MLPSpec(D, H, A), 2)
    r_v = ref.mlp_forward_ref(0, pv, X, A, H)
    g_v = mlp_forward(FwdMode.VALUE, pv.to(cuda), X.to(cuda), A, H)
    torch.testing.assert_close(g_v["v"].cpu(), r_v["v"], rtol=1e-4, atol=1e-5)
    r_l = ref.mlp_forward_ref(3, pp, X, A, H, mask=mask)
    g_l = mlp_forward(FwdMode.LOGITS, pp.to(cuda), X.to(cuda), A, H, mask=mask.to(cuda))
    torch.testing.assert_close(g_l["logits"].cpu(), r_l["logits"], rtol=1e-4, atol=1e-4)
    r_e = ref.mlp_forward_ref(2, pp, X, A, H, mask=mask, act_in=act)
    g_e = mlp_forward(FwdMode.CAT_EVAL, pp.to(cuda), X.to(cuda), A, H, mask=mask.to(cuda), act_in=act.to(cuda))
    torch.testing.assert_close(g_e["logp"].cpu(), r_e["logp"], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(g_e["entropy"].cpu(), r_e["entropy"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("D,H,A,B", SHAPES)
def test_forward_sample_matches_philox_oracle(cuda, D, H, A, B):
    torch.manual_seed(7 + B)
    X = torch.randn(B, D)
    pp = _params(MLPSpec(D, H, A), 3)
    seed, step, off = 1234567, 42, 100
    r = ref.mlp_forward_ref(1, pp, X, A, H, seed=seed, step=step, row_offset=off)
    g = mlp_forward(FwdMode.CAT_SAMPLE, pp.to(cuda), X.to(cuda), A, H, seed=seed, step=step, row_offset=off)
    mism = (g["act"].cpu() != r["act"]).float().mean().item()
    assert mism <= 0.01, mism  # only u within ~1e-6 of a cdf boundary may differ
    same = g["act"].cpu() == r["act"]
    torch.testing.assert_close(g["logp"].cpu()[same], r["logp"][same], rtol=1e-4, atol=1e-4)


def test_sample_distribution_chi2(cuda):
    # many rows with identical logits -> empirical frequencies match softmax
    D, H, A, B = 4, 128, 4, 200000
    pp = _params(MLPSpec(D, H, A), 5)
    X = torch.ones(B, D) * 0.3
    g = mlp_forward(FwdMode.CAT_SAMPLE, pp.to(cuda), X.to(cuda), A, H, seed=99, step=1)
    p = torch.softmax(ref.mlp_forward_ref(3, pp, X[:1], A, H)["logits"][0], -1).numpy()
    counts = np.bincount(g["act"].cpu().numpy(), minlength=A)
    exp = p * B
    chi2 = (((counts - exp) ** 2) / exp).sum()
    assert chi2 < 30.0, (counts, exp)


@pytest.mark.parametrize("D,H,A,B", [(4, 128, 2, 500), (17, 128, 6, 200), (3, 64, 2, 77)])
def test_forward_gaussian(cuda, D, H, A, B):
    torch.manual_seed(11)
    X = torch.randn(B, D)
    spec = MLPSpec(D, H, A, gaussian=True)
    pp = _params(spec, 4)
    r = ref.mlp_forward_ref(4, pp, X, A, H, seed=5, step=9)
    g = mlp_forward(FwdMode.GAUSS_SAMPLE, pp.to(cuda), X.to(cuda), A, H, seed=5, step=9)
    torch.testing.assert_close(g["act"].cpu(), r["act"], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(g["logp"].cpu(), r["logp"], rtol=1e-3, atol=2e-3)
    act = r["act"]
    r2 = ref.mlp_forward_ref(5, pp, X, A, H, actc_in=act)
    g2 = mlp_forward(FwdMode.GAUSS_EVAL, pp.to(cuda), X.to(cuda), A, H, actc_in=act.to(cuda))
    torch.testing.assert_close(g2["logp"].cpu(), r2["logp"], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(g2["entropy"].cpu(), r2["entropy"], rtol=1e-4, atol=1e-4)


GRAD_CASES = [
    (GradHead.PG_CAT, 4, 128, 2, 1000),
    (GradHead.PG_CAT, 8, 128, 4, 4100),
    (GradHead.PG_CAT, 17, 128, 6, 333),
    (GradHead.VALUE_MSE, 4, 128, 2, 1000),
    (GradHead.VALUE_MSE, 8, 64, 4, 70),
    (GradHead.PPO_CAT, 4, 128, 2, 2000),
    (GradHead.PPO_GAUSS, 17, 128, 6, 1500),
    (GradHead.PG_GAUSS, 5, 64, 3, 129),
    (GradHead.PG_GAUSS, 3, 128, 2, 700),
    (GradHead.VALUE_MSE, 4, 128, 1, 40000),   # several 64-row slabs per workgroup
    (GradHead.VALUE_MSE, 2, 128, 1, 777),     # D < 4, ragged tail
    (GradHead.VALUE_MSE, 3, 128, 1, 16),
    (GradHead.PG_CAT, 4, 128, 2, 40000),
]


@pytest.mark.parametrize("head,D,H,A,B", GRAD_CASES)
def test_grad_matches_autograd(cuda, head, D, H, A, B):
    torch.manual_seed(int(head) * 100 + B)
    gaussian = head in (GradHead.PPO_GAUSS, GradHead.PG_GAUSS)
    Aeff = 1 if head == GradHead.VALUE_MSE else A
    spec = MLPSpec(D, H, Aeff, gaussian)
    pp = _params(spec, 6)
    X = torch.randn(B, D)
    mask = None
    act = torch.randint(0, A, (B,), dtype=torch.int32)
    actc = torch.randn(B, A) * 0.5
    adv = torch.randn(B) * 2 + 0.3
    ret = torch.randn(B) * 3
    logp_old = -torch.rand(B) * 2 if not gaussian else -torch.rand(B) * 8
    stats = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(B))])
    kw = dict(act=act, actc=actc, adv=adv, ret=ret, logp_old=logp_old, adv_stats=stats, clip_eps=0.2, ent_coef=0.01)
    g_ref, st = ref.mlp_grad_ref(int(head), pp, X, A, H, mask, **kw)
    kwd = {k: (v.to(cuda) if torch.is_tensor(v) else v) for k, v in kw.items()}
    slab, loss = mlp_grad(head, pp.to(cuda), X.to(cuda), A, H, None, **kwd)
    g = slab.sum(0).cpu()
    scale = g_ref.abs().max().item() + 1e-12
    err = (g - g_ref).abs().max().item()
    assert err <= 2e-4 * scale + 1e-6, (err, scale)
    ls = loss.sum(0).cpu()
    assert abs(ls[0].item() - st["loss"]) <= 1e-3 * (abs(st["loss"]) + 1)
    assert int(ls[5].item()) == B


def test_grad_reduce_and_adam_match_torch(cuda):
    torch.manual_seed(0)
    D, H, A, B = 4, 128, 2, 3000
    spec = MLPSpec(D, H, A)
    p0 = _params(spec, 8)
    X = torch.randn(B, D)
    act = torch.randint(0, A, (B,), dtype=torch.int32)
    adv = torch.randn(B)
    # torch.optim.Adam oracle
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=3e-3)
    pg = p0.clone().to(cuda)
    m = torch.zeros_like(pg)
    v = torch.zeros_like(pg)
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    ticket = torch.zeros(1, dtype=torch.int32, device=cuda)
    for it in range(5):
        g_ref, _ = ref.mlp_grad_ref(0, pt.detach(), X, A, H, act=act, adv=adv)
        opt.zero_grad()
        pt.grad = g_ref.clone()
        opt.step()
        slab, _ = mlp_grad(GradHead.PG_CAT, pg, X.to(cuda), A, H, act=act.to(cuda), adv=adv.to(cuda))
        adam_step(pg, m, v, step, ticket, 3e-3, slab=slab)
    assert int(step.item()) == 5
    torch.testing.assert_close(pg.cpu(), pt.detach(), rtol=1e-4, atol=2e-6)
    red = reduce_slabs(slab, 0.5)
    torch.testing.assert_close(red.cpu(), slab.sum(0).cpu() * 0.5, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("nslab", [1, 5, 63, 64, 128, 129, 200, 256, 300])
def test_slab_reduction_and_adam_all_batchings(cuda, nslab):
    """The slab sum issues 8 loads, then 4, then single loads per thread: every path vs fp64."""
    torch.manual_seed(nslab)
    P = 17_000
    slab = torch.randn(nslab, P)
    ref_sum = slab.double().sum(0)
    red = reduce_slabs(slab.to(cuda), 1.0)
    torch.testing.assert_close(red.cpu().double(), ref_sum, rtol=1e-5, atol=1e-5)
    p0 = torch.randn(P)
    pg = p0.clone().to(cuda)
    m = torch.zeros_like(pg)
    v = torch.zeros_like(pg)
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    ticket = torch.zeros(1, dtype=torch.int32, device=cuda)
    adam_step(pg, m, v, step, ticket, 1e-3, slab=slab.to(cuda))
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=1e-3)
    pt.grad = ref_sum.float()
    opt.step()
    assert int(step.item()) == 1
    torch.testing.assert_close(pg.cpu(), pt.detach(), rtol=1e-5, atol=1e-6)


def test_adam_loop_form_of_the_step_counter(cuda):
    """A loop of K Adam updates passing (step_add, step_inc) = (k, 0) and (K - 1, K) last -- no
    arrival ticket but on the last update -- equals K single updates bitwise (same bias
    corrections), and leaves the counter at s0 + K; the CPU path agrees."""
    torch.manual_seed(3)
    P, K = 17_281, 6
    slabs = [torch.randn(7, P, device=cuda) for _ in range(K)]
    p0 = torch.randn(P, device=cuda)
    outs = []
    for loop in (False, True):
        pg, m, v = p0.clone(), torch.zeros(P, device=cuda), torch.zeros(P, device=cuda)
        step = torch.full((1,), 4, dtype=torch.int32, device=cuda)  # resumed after 4 updates
        ticket = torch.zeros(1, dtype=torch.int32, device=cuda)
        for k in range(K):
            if loop:
                adam_step(pg, m, v, step, ticket, 1e-3, slab=slabs[k], step_add=k, step_inc=K if k == K - 1 else 0)
            else:
                adam_step(pg, m, v, step, ticket, 1e-3, slab=slabs[k])
        torch.cuda.synchronize()
        assert int(step.item()) == 4 + K and int(ticket.item()) == 0
        outs.append((pg.clone(), m.clone(), v.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # the CPU (torch) path of the same loop
    pc, mc, vc = p0.cpu(), torch.zeros(P), torch.zeros(P)
    sc, tc = torch.full((1,), 4, dtype=torch.int32), torch.zeros(1, dtype=torch.int32)
    for k in range(K):
        adam_step(pc, mc, vc, sc, tc, 1e-3, slab=slabs[k].cpu(), step_add=k, step_inc=K if k == K - 1 else 0)
    assert int(sc.item()) == 4 + K
    torch.testing.assert_close(pc, outs[0][0].cpu(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("T,N,baseline", [(64, 1000, True), (128, 33, False), (7, 5000, True)])
def test_gae_scan_tm(cuda, T, N, baseline):
    torch.manual_seed(T + N)
    rew = torch.randn(T, N)
    done = (torch.rand(T, N) < 0.05).float()
    val = torch.randn(T + 1, N) if baseline else None
    a_r, r_r, s_r = ref.gae_scan_tm_ref(rew, done, val, 0.98, 0.97)
    a_g, r_g, s_g = gae_scan_tm(rew.to(cuda), done.to(cuda), None if val is None else val.to(cuda), 0.98, 0.97)
    torch.testing.assert_close(a_g.cpu(), a_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(r_g.cpu(), r_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(s_g.cpu(), s_r, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("L,baseline", [(1, True), (100, False), (5000, True), (70000, True), (70001, False)])
def test_scan_flat(cuda, L, baseline):
    torch.manual_seed(L)
    rew = torch.randn(L)
    done = (torch.rand(L) < 0.01).float()
    done[-1] = 1.0
    val = torch.randn(L) if baseline else None
    boot = torch.randn(L) if baseline else None
    a_r, r_r, s_r = ref.scan_flat_ref(rew, done, val, boot, 0.99, 0.95)
    a_g, r_g, s_g = scan_flat(rew.to(cuda), done.to(cuda), None if val is None else val.to(cuda),
                              None if boot is None else boot.to(cuda), 0.99, 0.95)
    torch.testing.assert_close(a_g.cpu(), a_r, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(r_g.cpu(), r_r, rtol=1e-3, atol=1e-3)
