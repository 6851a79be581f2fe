"""TorchScript-exportable policy modules (checkpoint / model-file compatibility).

The reference's model file is a TorchScript archive of ``PolicyWithoutBaseline`` /
``PolicyWithBaseline`` exposing ``step(obs, mask) -> (act, Dict[str, Tensor])``,
``get_input_dim()`` and ``get_output_dim()`` (kernel.py:87-143; validated by
agent_wrapper.rs:88-168).  These modules rebuild that interface from our flat fp32
parameter vectors (same Linear order, so ``data/0..5`` hold W1,b1,W2,b2,W3,b3) with the
documented fixes: ``logp_a`` is the true log_softmax (kernel.py:33-37 gathered the raw
logit), and the Gaussian policy is complete (kernel.py:49-75 was a stub).

On the GPU hot path none of this runs -- the fused HIP kernels read the flat vector.
"""
from __future__ import annotations

from typing import Any, Dict, List, Tuple

import torch
import torch.nn as nn

from ..ops.mlp import MLPSpec


def mlp(sizes: List[int], activation=nn.ReLU, output_activation=nn.Identity) -> nn.Sequential:
    """BaseKernel.mlp (BaseKernel.py:25-39)."""
    layers = []
    for j in range(len(sizes) - 1):
        act = activation if j < len(sizes) - 2 else output_activation
        layers += [nn.Linear(sizes[j], sizes[j + 1]), act()]
    return nn.Sequential(*layers)


class DiscretePolicyNetwork(nn.Module):
    def __init__(self, obs_dim: int, hidden_sizes: List[int], act_dim: int):
        super().__init__()
        self.pi_network = mlp([obs_dim] + list(hidden_sizes) + [act_dim])

    def distribution(self, obs: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        logits = self.pi_network(obs)
        logits = logits + (mask - 1.0) * 1e8
        return torch.softmax(logits, dim=-1), torch.log_softmax(logits, dim=-1)

    def sample(self, obs: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        probs, logp_all = self.distribution(obs, mask)
        flat = probs.reshape(-1, probs.shape[-1])
        act = torch.multinomial(flat, 1).reshape(probs.shape[:-1] + (1,))
        return act, logp_all.gather(-1, act).squeeze(-1)

    def forward(self, obs: torch.Tensor, mask: torch.Tensor, act: torch.Tensor):
        probs, logp_all = self.distribution(obs, mask)
        logp_a = logp_all.gather(-1, act.long().unsqueeze(-1)).squeeze(-1)
        return probs, logp_all, logp_a


class ContinuousPolicyNetwork(nn.Module):
    def __init__(self, obs_dim: int, hidden_sizes: List[int], act_dim: int, log_std_init: float = -0.5):
        super().__init__()
        self.pi_network = mlp([obs_dim] + list(hidden_sizes) + [act_dim])
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))

    def sample(self, obs: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        mu = self.pi_network(obs)
        std = torch.exp(self.log_std)
        a = mu + std * torch.randn_like(mu)
        z = (a - mu) / std
        return a, (-0.5 * z * z - self.log_std - 0.9189385332046727).sum(-1)

    def forward(self, obs: torch.Tensor, mask: torch.Tensor, act: torch.Tensor):
        mu = self.pi_network(obs)
        std = torch.exp(self.log_std)
        z = (act - mu) / std
        logp = (-0.5 * z * z - self.log_std - 0.9189385332046727).sum(-1)
        return mu, std, logp


class BaselineValueNetwork(nn.Module):
    def __init__(self, obs_dim: int, hidden_sizes: List[int]):
        super().__init__()
        self.v_network = mlp([obs_dim] + list(hidden_sizes) + [1])

    def forward(self, obs: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        return self.v_network(obs).squeeze(-1)


class PolicyWithoutBaseline(nn.Module):
    def __init__(self, obs_dim: int, act_dim: int, discrete: bool = True, hidden_sizes: List[int] = (128, 128)):
        super().__init__()
        self.discrete = discrete
        if discrete:
            self.policy = DiscretePolicyNetwork(obs_dim, list(hidden_sizes), act_dim)
        else:
            self.policy = ContinuousPolicyNetwork(obs_dim, list(hidden_sizes), act_dim)
        self.input_dim = obs_dim
        self.output_dim = act_dim

    def _act(self, obs: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.policy.sample(obs, mask)

    @torch.jit.export
    def step(self, obs: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        with torch.no_grad():
            act, logp = self._act(obs, mask)
        data: Dict[str, torch.Tensor] = {"logp_a": logp}
        return act, data

    @torch.jit.export
    def get_input_dim(self) -> int:
        return self.input_dim

    @torch.jit.export
    def get_output_dim(self) -> int:
        return self.output_dim


class PolicyWithBaseline(PolicyWithoutBaseline):
    def __init__(self, obs_dim: int, act_dim: int, discrete: bool = True, hidden_sizes: List[int] = (128, 128)):
        super().__init__(obs_dim, act_dim, discrete, hidden_sizes)
        self.baseline = BaselineValueNetwork(obs_dim, list(hidden_sizes))

    @torch.jit.export
    def step(self, obs: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        with torch.no_grad():
            act, logp = self._act(obs, mask)
            v = self.baseline(obs, mask)
        data: Dict[str, torch.Tensor] = {"logp_a": logp, "v": v}
        return act, data


def _load_linear_stack(seq: nn.Sequential, params: torch.Tensor, spec: MLPSpec):
    W1, b1, W2, b2, W3, b3, log_std = spec.unflatten(params.detach().float().cpu())
    lin = [m for m in seq if isinstance(m, nn.Linear)]
    with torch.no_grad():
        for m, (w, b) in zip(lin, ((W1, b1), (W2, b2), (W3, b3))):
            m.weight.copy_(w)
            m.bias.copy_(b)
    return log_std


def build_policy_module(obs_dim: int, act_dim: int, hidden: int, pi_params: torch.Tensor, vf_params=None,
                        discrete: bool = True) -> nn.Module:
    """nn.Module (TorchScript-able) with the weights of the flat parameter vectors."""
    if vf_params is None:
        m = PolicyWithoutBaseline(obs_dim, act_dim, discrete, [hidden, hidden])
    else:
        m = PolicyWithBaseline(obs_dim, act_dim, discrete, [hidden, hidden])
        _load_linear_stack(m.baseline.v_network, vf_params, MLPSpec(obs_dim, hidden, 1))
    log_std = _load_linear_stack(m.policy.pi_network, pi_params, MLPSpec(obs_dim, hidden, act_dim, not discrete))
    if not discrete:
        with torch.no_grad():
            m.policy.log_std.copy_(log_std)
    return m.eval()


def flat_from_module(m: nn.Module, discrete: bool = True):
    """Inverse of build_policy_module -> (pi_params, vf_params or None).

    Works on eager and scripted modules (reads the state dict, in Linear order)."""
    sd = m.state_dict()

    def flat(prefix):
        parts = []
        for i in (0, 2, 4):
            parts += [sd[f"{prefix}.{i}.weight"].reshape(-1), sd[f"{prefix}.{i}.bias"].reshape(-1)]
        return parts

    pi = flat("policy.pi_network")
    if "policy.log_std" in sd:
        pi.append(sd["policy.log_std"].reshape(-1))
    vf = torch.cat(flat("baseline.v_network")).float() if "baseline.v_network.0.weight" in sd else None
    return torch.cat(pi).float(), vf


def module_dims(m: nn.Module):
    """(obs_dim, act_dim, hidden, discrete) of an exported policy module."""
    sd = m.state_dict()
    w1 = sd["policy.pi_network.0.weight"]
    w3 = sd["policy.pi_network.4.weight"]
    return int(w1.shape[1]), int(w3.shape[0]), int(w1.shape[0]), "policy.log_std" not in sd


# TorchScript qualified names of the reference model file: the archive holds
# code/__torch__/REINFORCE/kernel.py with class PolicyWithoutBaseline / PolicyWithBaseline
# (examples/.../cartpole/zmq/client_model.pt; REINFORCE.py:64-68 scripts kernel.py's classes).
# Export-only subclasses carry that module path; the exported copy's submodules are re-classed
# to them just before scripting (TorchScript caches compiled types per Python class, so the
# working classes keep their own names).
REFERENCE_MODULE = "REINFORCE.kernel"
_REF_CLASSES = {base: type(base.__name__, (base,), {"__module__": REFERENCE_MODULE, "__qualname__": base.__name__})
                for base in (DiscretePolicyNetwork, ContinuousPolicyNetwork, BaselineValueNetwork,
                             PolicyWithoutBaseline, PolicyWithBaseline)}


def reference_named(module: nn.Module) -> nn.Module:
    """A copy of ``module`` whose policy classes script as ``__torch__.REINFORCE.kernel.*``."""
    import copy

    m = copy.deepcopy(module)
    for sub in m.modules():
        cls = _REF_CLASSES.get(type(sub))
        if cls is not None:
            sub.__class__ = cls
    return m


def _save_scripted(module: nn.Module, path: str) -> None:
    torch.jit.save(torch.jit.script(reference_named(module)), path)


def export_torchscript(module: nn.Module, path: str) -> None:
    """torch.jit.script + save (REINFORCE.py:64-68), written atomically.  The archive root is
    the file's stem (``server_model/`` for server_model.pt, like the reference), so the file is
    written under its final name inside a private temp directory and then moved."""
    import os
    import tempfile

    d = tempfile.mkdtemp(prefix=".rrl_export_", dir=os.path.dirname(os.path.abspath(path)))
    try:
        tmp = os.path.join(d, os.path.basename(path))
        _save_scripted(module, tmp)
        os.replace(tmp, path)
    finally:
        try:
            os.rmdir(d)
        except OSError:
            pass


def torchscript_bytes(module: nn.Module, archive: str = "server_model") -> bytes:
    """The TorchScript archive as bytes, rooted at ``{archive}/`` (reference: server_model/)."""
    import os
    import tempfile

    with tempfile.TemporaryDirectory(prefix="rrl_ts_") as d:
        path = os.path.join(d, f"{archive}.pt")
        _save_scripted(module, path)
        with open(path, "rb") as f:
            return f.read()


_SCRIPTED: Dict[tuple, Any] = {}
_SCRIPTED_LOCK = __import__("threading").Lock()


def torchscript_bytes_flat(obs_dim: int, act_dim: int, hidden: int, pi_params, vf_params=None,
                           discrete: bool = True, archive: str = "server_model") -> bytes:
    """``torchscript_bytes(build_policy_module(...))`` without re-scripting: one scripted module
    per layout is compiled once and each version's flat weights are copied into it before the
    save.  Same archive (classes ``__torch__.REINFORCE.kernel.*``, root ``{archive}/``); ~30x
    less work per published version, which matters because the export runs on a transport's
    publisher thread next to the learner (GIL)."""
    import os
    import tempfile

    pi = torch.as_tensor(pi_params, dtype=torch.float32)
    vf = None if vf_params is None else torch.as_tensor(vf_params, dtype=torch.float32)
    key = (int(obs_dim), int(act_dim), int(hidden), bool(discrete), vf is not None)
    with _SCRIPTED_LOCK:
        sm = _SCRIPTED.get(key)
        if sm is None:
            sm = torch.jit.script(reference_named(build_policy_module(obs_dim, act_dim, hidden, pi, vf, discrete)))
            _SCRIPTED[key] = sm
        else:
            fresh = build_policy_module(obs_dim, act_dim, hidden, pi, vf, discrete).state_dict()
            with torch.no_grad():
                for k, t in sm.state_dict().items():
                    t.copy_(fresh[k])
        with tempfile.TemporaryDirectory(prefix="rrl_ts_") as d:
            path = os.path.join(d, f"{archive}.pt")
            torch.jit.save(sm, path)
            with open(path, "rb") as f:
                return f.read()
