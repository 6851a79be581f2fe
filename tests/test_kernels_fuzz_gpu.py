"""Shape fuzzing (hypothesis) of the fused MLP kernels against the fp32 oracle on the GPU:
random obs / action dims, hidden sizes and batch sizes (including batches that are not
multiples of the 16-row tiles or of the 64-row staging images)."""
import pytest
import torch
from hypothesis import HealthCheck, assume, given, settings
from hypothesis import strategies as st

from relayrl_prototype_amd.ops import FwdMode, GradHead, MLPSpec, mlp_forward, mlp_grad
from relayrl_prototype_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
FUZZ = settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                       HealthCheck.function_scoped_fixture])


@FUZZ
@given(D=st.integers(1, 32), A=st.integers(1, 8), H=st.sampled_from([64, 128]), B=st.integers(1, 700),
       seed=st.integers(0, 10 ** 6))
def test_forward_logits_value_fuzz(cuda, D, A, H, B, seed):  # D up to 32: two input tiles
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(B, D, generator=g)
    pp = MLPSpec(D, H, A).init(g)
    pv = MLPSpec(D, H, 1).init(g)
    r = ref.mlp_forward_ref(3, pp, X, A, H)
    k = mlp_forward(FwdMode.LOGITS, pp.to(cuda), X.to(cuda), A, H)
    torch.testing.assert_close(k["logits"].cpu(), r["logits"], rtol=1e-4, atol=1e-4)
    rv = ref.mlp_forward_ref(0, pv, X, A, H)
    kv = mlp_forward(FwdMode.VALUE, pv.to(cuda), X.to(cuda), A, H)
    torch.testing.assert_close(kv["v"].cpu(), rv["v"], rtol=1e-4, atol=1e-4)


@FUZZ
@given(head=st.sampled_from([GradHead.PG_CAT, GradHead.VALUE_MSE, GradHead.PPO_CAT]), D=st.integers(1, 32),
       A=st.integers(2, 8), H=st.sampled_from([64, 128]), B=st.integers(1, 700), seed=st.integers(0, 10 ** 6))
def test_grad_fuzz(cuda, head, D, A, H, B, seed):
    g = torch.Generator().manual_seed(seed)
    Aeff = 1 if head == GradHead.VALUE_MSE else A
    sp = MLPSpec(D, H, Aeff)
    pp = sp.init(g)
    X = torch.randn(B, D, generator=g)
    # a ReLU tie (|pre-activation| ~ rounding) flips relu' between two correct fp32 evaluation
    # orders and moves a whole dW2 / b2 row: not a kernel error (seed 1000000, D 1, A 5, B 45:
    # |z2| = 9.6e-9 against a median of 0.2, tools/grad_fuzz_probe.py)
    o = sp.offsets()
    p64, x64 = pp.double(), X.double()
    z1 = x64 @ p64[o["w1"]:o["b1"]].view(H, D).T + p64[o["b1"]:o["w2"]]
    z2 = z1.clamp(min=0) @ p64[o["w2"]:o["b2"]].view(H, H).T + p64[o["b2"]:o["w3"]]
    assume(min(z1.abs().min().item(), z2.abs().min().item()) > 1e-6)
    act = torch.randint(0, A, (B,), dtype=torch.int32, generator=g)
    adv = torch.randn(B, generator=g)
    ret = torch.randn(B, generator=g)
    logp_old = -torch.rand(B, generator=g) * 2
    stats = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(B))])
    kw = dict(act=act, adv=adv, ret=ret, logp_old=logp_old, adv_stats=stats, clip_eps=0.2, ent_coef=0.01)
    g_ref, _ = ref.mlp_grad_ref(int(head), pp, X, A, H, None, **kw)
    slab, _ = mlp_grad(head, pp.to(cuda), X.to(cuda), A, H, None,
                       **{k: (v.to(cuda) if torch.is_tensor(v) else v) for k, v in kw.items()})
    gk = slab.sum(0).cpu()
    scale = g_ref.abs().max().item() + 1e-12
    assert (gk - g_ref).abs().max().item() / scale < 2e-4
