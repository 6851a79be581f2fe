"""Native checkpoint / resume.

The reference persisted only the TorchScript policy (server_model.pt / client_model.pt);
optimizer state, counters and RNG were lost, so there was no real resume.  Here a
checkpoint directory holds:

  tensors.safetensors  -- every tensor of the trainer/algorithm state (flat params,
                          Adam m / v / step, env state for the vectorised trainer)
  state.json           -- scalars (epoch, env steps, versions, config snapshot)
  model.pt             -- optional TorchScript export for agents (compat format)

``import_reference_weights`` reads the raw fp32 storages (data/0..5) of a reference
TorchScript archive with ``zipfile`` -- nothing from the file is unpickled or executed.
"""
from __future__ import annotations

import json
import os
import tempfile
import zipfile
from typing import Any, Dict, Tuple

import numpy as np
import torch

SEP = "/"


def _flatten(d: Dict[str, Any], prefix: str = ""):
    tensors, scalars = {}, {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            t, s = _flatten(v, key + SEP)
            tensors.update(t)
            scalars.update(s)
        elif torch.is_tensor(v):
            tensors[key] = v.detach().cpu().contiguous()
        elif isinstance(v, np.ndarray):
            tensors[key] = torch.from_numpy(np.ascontiguousarray(v))
        else:
            scalars[key] = v
    return tensors, scalars


def _unflatten(tensors: Dict[str, torch.Tensor], scalars: Dict[str, Any]) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for src in (scalars, tensors):
        for k, v in src.items():
            parts = k.split(SEP)
            cur = out
            for p in parts[:-1]:
                cur = cur.setdefault(p, {})
            cur[parts[-1]] = v
    return out


def save_checkpoint(directory: str, state: Dict[str, Any], model_module=None) -> str:
    from safetensors.torch import save_file

    os.makedirs(directory, exist_ok=True)
    tensors, scalars = _flatten(state)
    tmp = tempfile.mkdtemp(dir=directory)
    save_file(tensors, os.path.join(tmp, "tensors.safetensors"))
    with open(os.path.join(tmp, "state.json"), "w") as f:
        json.dump(scalars, f, indent=1, sort_keys=True, default=str)
    for name in ("tensors.safetensors", "state.json"):
        os.replace(os.path.join(tmp, name), os.path.join(directory, name))
    os.rmdir(tmp)
    if model_module is not None:
        from ..models.policies import export_torchscript

        export_torchscript(model_module, os.path.join(directory, "model.pt"))
    return directory


def load_checkpoint(directory: str) -> Dict[str, Any]:
    from safetensors.torch import load_file

    tensors = load_file(os.path.join(directory, "tensors.safetensors"))
    with open(os.path.join(directory, "state.json")) as f:
        scalars = json.load(f)
    return _unflatten(tensors, scalars)


def periodic_checkpointer(directory: str, every: int):
    """LearnerService hook: checkpoint the algorithm every ``every`` model updates."""

    def fn(service):
        if service.updates % every == 0:
            alg = service.algorithm
            save_checkpoint(os.path.join(directory, "latest"), alg.state_dict())

    return fn


def import_reference_weights(pt_path: str, obs_dim: int, act_dim: int, hidden: int = 128) -> Tuple[np.ndarray, ...]:
    """Flat fp32 (pi_params, vf_params|None) from a reference TorchScript archive.

    The archive's ``data/N`` entries are raw little-endian storages; for
    PolicyWithoutBaseline they are W1,b1,W2,b2,W3,b3 (2048/512/65536/512/
    1024/8 B for CartPole).  Storages are matched to the Linear layout by byte size.
    """
    D, H, A = obs_dim, hidden, act_dim
    pi_sizes = [H * D, H, H * H, H, A * H, A]
    vf_sizes = [H * D, H, H * H, H, H, 1]
    with zipfile.ZipFile(pt_path) as z:
        entries = {}
        for n in z.namelist():
            parts = n.split("/")
            if len(parts) >= 2 and parts[-2] == "data" and parts[-1].isdigit():
                entries[int(parts[-1])] = np.frombuffer(z.read(n), dtype="<f4").copy()
    order = [entries[k] for k in sorted(entries)]
    sizes = [a.size for a in order]
    if sizes[:6] != pi_sizes:
        raise ValueError(f"storage sizes {sizes} do not match a [{D},{H},{H},{A}] policy")
    pi = np.concatenate(order[:6]).astype(np.float32)
    vf = None
    if len(order) >= 12 and sizes[6:12] == vf_sizes:
        vf = np.concatenate(order[6:12]).astype(np.float32)
    return pi, vf


def reference_weights_from_bytes(blob: bytes) -> Dict[str, Any]:
    """A TorchScript policy archive as the reference server pushes it (training_zmq.rs:876-934,
    agent_zmq.rs:625-698: the bytes of ``torch.jit.save`` of PolicyWithoutBaseline /
    PolicyWithBaseline, kernel.py:87-143) -> flat fp32 weights and the dims, read from the
    zip's raw ``data/N`` storages only (the archive's pickles are never executed).

    The dims come from the storage sizes of the Linear stack [H*D, H, H*H, H, A*H, A]
    (+ the value net's [H*D, H, H*H, H, H, 1] for PolicyWithBaseline)."""
    import io

    import re

    acts = set()
    with zipfile.ZipFile(io.BytesIO(blob)) as z:
        entries = {}
        for n in z.namelist():
            parts = n.split("/")
            if len(parts) >= 2 and parts[-2] == "data" and parts[-1].isdigit():
                entries[int(parts[-1])] = np.frombuffer(z.read(n), dtype="<f4").copy()
            elif n.endswith("/torch/nn/modules/activation.py"):  # TorchScript source text, read not run
                acts |= set(re.findall(r"^class (\w+)\(", z.read(n).decode("utf-8", "replace"), re.M))
    order = [entries[k] for k in sorted(entries)]
    # the layout is recognised only when it is exactly ours: ReLU activations and 6 (policy) or
    # 12 (policy + baseline) storages -- anything else (a plugin's tanh net, extra parameters)
    # is an arbitrary TorchScript model that the agent runs through its step()
    if acts - {"ReLU"}:
        raise ValueError(f"activations {sorted(acts)} are not the ReLU MLP layout")
    if len(order) not in (6, 12):
        raise ValueError(f"a policy archive holds 6 or 12 storages, found {len(order)}")
    s = [a.size for a in order]
    H = s[1]
    if H < 1 or s[0] % H or s[2] != H * H or s[3] != H or s[4] % H or s[5] * H != s[4]:
        raise ValueError(f"storage sizes {s[:6]} are not a Linear-ReLU-Linear-ReLU-Linear policy")
    D = s[0] // H
    value_sizes = [H * D, H, H * H, H, H, 1]
    first, second = order[:6], order[6:12]
    if len(order) >= 12 and s[:6] == value_sizes and s[6:12] != value_sizes:
        first, second = second, first  # a module that lists its baseline before its policy
    sf = [a.size for a in first]
    A = sf[5]
    if sf != [H * D, H, H * H, H, A * H, A]:
        raise ValueError(f"storage sizes {sf} are not a [{D}, {H}, {H}, A] policy")
    pi = np.concatenate(first).astype(np.float32)
    vf = None
    if len(second) == 6:
        if [a.size for a in second] != value_sizes:
            raise ValueError(f"storage sizes {[a.size for a in second]} are not a [{D}, {H}, {H}, 1] baseline")
        vf = np.concatenate(second).astype(np.float32)
    return {"pi": pi, "vf": vf, "obs_dim": int(D), "act_dim": int(A), "hidden": int(H)}
