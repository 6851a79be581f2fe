"""Algorithm registry + custom-plugin loader.

Built-ins: REINFORCE, PPO, A2C.  Custom algorithms follow the reference contract
(python_algorithm_reply.py:16-52): ``<algorithm_dir>/<NAME>/<NAME>.py`` defines class
``<NAME>``; it is imported in-process (no subprocess / JSON pipe) and constructed with
``env_dir, config_path, obs_dim, act_dim, buf_size`` plus the hyperparameter overrides
it accepts (unknown overrides are dropped with a warning instead of crashing, A9).
"""
from __future__ import annotations

import importlib
import inspect
import os
import sys
from typing import Any, Dict, Optional

from .ppo import A2C, PPO
from .reinforce import REINFORCE

BUILTINS = {"REINFORCE": REINFORCE, "PPO": PPO, "A2C": A2C}


def _coerce(v):
    """Hyperparameter strings from the CLI / list form -> numbers / bools."""
    if not isinstance(v, str):
        return v
    lo = v.strip().lower()
    if lo in ("true", "false"):
        return lo == "true"
    try:
        return int(v)
    except ValueError:
        pass
    try:
        return float(v)
    except ValueError:
        return v


def parse_hyperparams(hp) -> Dict[str, Any]:
    """dict[str, str] or list of "k=v" / "k v" strings (training_server_wrapper.rs:118-154)."""
    if hp is None:
        return {}
    if isinstance(hp, dict):
        return {str(k): _coerce(v) for k, v in hp.items()}
    out = {}
    for item in hp:
        item = str(item)
        if "=" in item:
            k, v = item.split("=", 1)
        elif " " in item.strip():
            k, v = item.strip().split(None, 1)
        else:
            raise ValueError(f"bad hyperparameter entry {item!r} (expected k=v or 'k v')")
        out[k.strip()] = _coerce(v.strip())
    return out


def load_algorithm_class(name: str, algorithm_dir: Optional[str] = None):
    if algorithm_dir:
        path = os.path.join(algorithm_dir, name, name + ".py")
        if os.path.exists(path):
            from .compat import install_reference_aliases

            install_reference_aliases()  # _common._algorithms.* / utils.logger import paths
            if algorithm_dir not in sys.path:
                sys.path.insert(0, algorithm_dir)
            mod = importlib.import_module(f"{name}.{name}")
            return getattr(mod, name)
    if name.upper() in BUILTINS:
        return BUILTINS[name.upper()]
    raise ValueError(f"unknown algorithm {name!r} (builtins: {list(BUILTINS)}; algorithm_dir={algorithm_dir!r})")


def make_algorithm(name: str, algorithm_dir: Optional[str] = None, **kwargs):
    cls = load_algorithm_class(name, algorithm_dir)
    sig = inspect.signature(cls.__init__)
    accepts_var_kw = any(p.kind == p.VAR_KEYWORD for p in sig.parameters.values())
    if not accepts_var_kw:
        dropped = [k for k in kwargs if k not in sig.parameters]
        if dropped:
            print(f"[registry] {name}: ignoring unsupported hyperparameters {dropped}", flush=True)
        kwargs = {k: v for k, v in kwargs.items() if k in sig.parameters}
    return cls(**kwargs)
