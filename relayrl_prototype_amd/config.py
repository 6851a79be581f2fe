"""``relayrl_config.json`` loader with the reference's exact defaults and fallbacks.

Reference: relayrl_framework/src/sys_utils/config_loader.rs (schema :121-222, defaults
:66-113, fallbacks :397-554) and its Python binding o3_config_loader.rs:41-212.

Semantics kept on purpose:
  * a missing file is created with DEFAULT_CONFIG_CONTENT when resolved through
    ``resolve_config_json_path`` (TrainingServer / RelayRLAgent / default path);
  * an unparseable file (or a section with the wrong shape -- serde fails the whole
    document) means every section falls back;
  * per-field fallbacks differ from the file defaults (REINFORCE block, server host "*"
    with ports 7776/7777/7778, client/server model paths swapped, TB params);
  * ``scalar_tags`` is split on ';'.
Deliberate extensions (documented in docs/COMPAT.md):
  * ``training_tensorboard`` is also accepted at the top level (default_config.json:39-45);
  * PPO and A2C parameter blocks are loaded (the reference whitelists PPO but returns None);
  * a namespaced ``"mi355x"`` block carries the device runtime settings.
"""
from __future__ import annotations

import copy
import json
import os
from typing import Any, Dict, Optional

DEFAULT_CONFIG_FILENAME = "relayrl_config.json"

DEFAULT_CONFIG_CONTENT = """{
    "algorithms": {
        "REINFORCE": {
            "discrete": true,
            "with_vf_baseline": false,
            "seed": 1,
            "traj_per_epoch": 8,
            "gamma": 0.98,
            "lam": 0.97,
            "pi_lr": 3e-4,
            "vf_lr": 1e-3,
            "train_vf_iters": 80
        }
    },
    "grpc_idle_timeout": 30,
    "max_traj_length": 1000,
    "model_paths": {
        "client_model": "client_model.pt",
        "server_model": "server_model.pt"
    },
    "server": {
        "_comment": "gRPC uses only this address (prefix is unused).",
        "training_server": {
            "prefix": "tcp://",
            "host": "127.0.0.1",
            "port": "50051"
        },
        "trajectory_server": {
            "prefix": "tcp://",
            "host": "127.0.0.1",
            "port": "7776"
        },
        "agent_listener": {
            "prefix": "tcp://",
            "host": "127.0.0.1",
            "port": "7777"
        }
    },
    "tensorboard": {
        "training_tensorboard": {
            "_comment1": "Runs `tensorboard --logdir /logs` in cwd on start up of server.",
            "launch_tb_on_startup": true,
            "_comment2": "scalar tags can be any column header from `progress.txt` files.",
            "scalar_tags": "AverageEpRet;LossQ",
            "global_step_tag": "Epoch"
        }
    }
}"""

AVAILABLE_ALGORITHMS = ("C51", "DDPG", "DQN", "PPO", "REINFORCE", "SAC", "TD3", "A2C")

# config_loader.rs:412-422 -- NOTE: differs from the file defaults on purpose.
REINFORCE_FALLBACK = {
    "discrete": True,
    "with_vf_baseline": True,
    "seed": 0,
    "traj_per_epoch": 12,
    "gamma": 0.99,
    "lam": 0.97,
    "pi_lr": 3e-4,
    "vf_lr": 1e-3,
    "train_vf_iters": 80,
}
PPO_FALLBACK = {
    "discrete": True,
    "seed": 0,
    "traj_per_epoch": 12,
    "gamma": 0.99,
    "lam": 0.95,
    "clip_ratio": 0.2,
    "pi_lr": 3e-4,
    "vf_lr": 1e-3,
    "train_pi_iters": 80,
    "train_vf_iters": 80,
    "target_kl": 0.01,
    "ent_coef": 0.0,
}
A2C_FALLBACK = {
    "discrete": True,
    "seed": 0,
    "traj_per_epoch": 12,
    "gamma": 0.99,
    "lam": 1.0,
    "pi_lr": 7e-4,
    "vf_lr": 7e-4,
    "train_vf_iters": 1,
    "ent_coef": 0.01,
}
ALGO_FALLBACKS = {"REINFORCE": REINFORCE_FALLBACK, "PPO": PPO_FALLBACK, "A2C": A2C_FALLBACK}

MI355X_DEFAULTS = {
    "world_size": 1,
    "envs_per_actor": 4096,
    "rollout_len": 128,
    "hidden": 128,
    "dtype": "fp32",
    "use_graphs": True,
    "transport": "rccl",
    "mode": "dp",  # dp | actor_learner
    "agent_timeout_s": 120.0,  # evict agents silent this long (0 = never); agents heartbeat every 10 s
    "agent_sweep_period_s": 5.0,
}

_REINFORCE_TYPES = {
    "discrete": bool,
    "with_vf_baseline": bool,
    "seed": int,
    "traj_per_epoch": int,
    "gamma": (int, float),
    "lam": (int, float),
    "pi_lr": (int, float),
    "vf_lr": (int, float),
    "train_vf_iters": int,
}


def _log(msg: str) -> None:
    if os.environ.get("RRL_QUIET_CONFIG") != "1":
        print(msg, flush=True)


def get_or_create_config_json_path(path: str) -> Optional[str]:
    """config_loader.rs:30-58: return the path, writing the default file if missing."""
    if os.path.exists(path):
        return path
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            f.write(DEFAULT_CONFIG_CONTENT)
        _log(f"[ConfigLoader - load_config] Created new config at: {path!r}")
        return path
    except OSError as e:
        _log(f"[ConfigLoader - load_config] Failed to create config file: {e}")
        return None


def default_config_path() -> Optional[str]:
    return get_or_create_config_json_path(os.path.join(os.getcwd(), DEFAULT_CONFIG_FILENAME))


def resolve_config_json_path(path: Optional[str]) -> Optional[str]:
    """The ``resolve_config_json_path!`` macro: explicit path (created if missing) or default."""
    if path is None:
        return default_config_path()
    if os.path.isdir(path):
        path = os.path.join(path, DEFAULT_CONFIG_FILENAME)
    return get_or_create_config_json_path(path)


def _is_type(v, t) -> bool:
    if t is int:
        return isinstance(v, int) and not isinstance(v, bool) and v >= 0
    if t is bool:
        return isinstance(v, bool)
    if isinstance(t, tuple):
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return isinstance(v, t)


def _server_ok(sp) -> bool:
    return isinstance(sp, dict) and all(isinstance(sp.get(k), str) for k in ("prefix", "host", "port"))


def _validate(cfg: Dict[str, Any]) -> bool:
    """Mimic serde: a present section with the wrong shape fails the whole document."""
    if not isinstance(cfg, dict):
        return False
    algos = cfg.get("algorithms")
    if algos is not None:
        if not isinstance(algos, dict):
            return False
        r = algos.get("REINFORCE")
        if r is not None:
            if not isinstance(r, dict):
                return False
            for k, t in _REINFORCE_TYPES.items():
                if k not in r or not _is_type(r[k], t):
                    return False
    srv = cfg.get("server")
    if srv is not None:
        if not isinstance(srv, dict):
            return False
        for k in ("training_server", "trajectory_server", "agent_listener"):
            if srv.get(k) is not None and not _server_ok(srv[k]):
                return False
    tb = cfg.get("tensorboard")
    if tb is not None:
        if not isinstance(tb, dict):
            return False
        p = tb.get("training_tensorboard")
        if p is not None and not _tb_ok(p):
            return False
    mp = cfg.get("model_paths")
    if mp is not None:
        if not isinstance(mp, dict):
            return False
        for k in ("client_model", "server_model"):
            if mp.get(k) is not None and not isinstance(mp[k], str):
                return False
    for k in ("max_traj_length", "grpc_idle_timeout"):
        if cfg.get(k) is not None and not _is_type(cfg[k], int):
            return False
    return True


def _tb_ok(p) -> bool:
    return (isinstance(p, dict) and isinstance(p.get("launch_tb_on_startup"), bool)
            and isinstance(p.get("scalar_tags"), str) and isinstance(p.get("global_step_tag"), str))


def load_config(path: Optional[str]) -> Dict[str, Any]:
    """config_loader.rs:308-341: unreadable / unparseable -> every section missing."""
    if path is None:
        return {}
    try:
        with open(path) as f:
            text = f.read()
    except OSError as e:
        _log(f"[ConfigLoader - load_config] Failed to load configuration from {path!r}, loading defaults. Error: {e}")
        return {}
    try:
        cfg = json.loads(text)
    except ValueError:
        _log("[ConfigLoader - load_config] Failed to parse configuration, loading empty defaults...")
        return {}
    if not _validate(cfg):
        _log("[ConfigLoader - load_config] Failed to parse configuration, loading empty defaults...")
        return {}
    return cfg


class ConfigLoader:
    """Python API identical to the reference's PyConfigLoader (o3_config_loader.rs:41-212)."""

    def __init__(self, algorithm_name: Optional[str] = None, config_path: Optional[str] = None):
        if config_path is None:
            config_path = default_config_path()
        elif os.path.isdir(config_path):
            config_path = os.path.join(config_path, DEFAULT_CONFIG_FILENAME)
        self.config_path = config_path
        self._cfg = load_config(config_path)
        self.algorithm_name = algorithm_name
        self.algorithm_params = self._set_algorithm_params(algorithm_name) if algorithm_name else None
        srv = self._cfg.get("server") or {}
        self.train_server = self._server(srv.get("training_server"), "7776", "training server")
        self.traj_server = self._server(srv.get("trajectory_server"), "7777", "trajectory server")
        self.agent_listener = self._server(srv.get("agent_listener"), "7778", "agent listener")
        self.grpc_idle_timeout = self._cfg.get("grpc_idle_timeout", 30)
        self.tb_params = self._set_tb_params()
        cwd = os.getcwd()
        mp = self._cfg.get("model_paths") or {}
        self.client_model_path = os.path.join(cwd, mp.get("client_model") or "server_model.pt")  # swap: :504-518
        self.server_model_path = os.path.join(cwd, mp.get("server_model") or "client_model.pt")  # swap: :520-534
        self.max_traj_length = self._cfg.get("max_traj_length", 1000)
        m = copy.deepcopy(MI355X_DEFAULTS)
        if isinstance(self._cfg.get("mi355x"), dict):
            m.update(self._cfg["mi355x"])
        self.mi355x = m

    # ------------------------------------------------------------------ setters
    def _set_algorithm_params(self, algo: str):
        block = (self._cfg.get("algorithms") or {}).get(algo)
        if algo not in AVAILABLE_ALGORITHMS and isinstance(block, dict):
            # a custom plugin's own block (rf/README.md:231-253): returned as written
            return {algo: {k: v for k, v in block.items() if not k.startswith("_")}}
        if algo not in AVAILABLE_ALGORITHMS:
            _log("[ConfigLoader - set_algorithm_params] Failed to load algorithm hyperparameters, loading defaults...")
            return None
        if algo not in ALGO_FALLBACKS:
            _log(f"[ConfigLoader - set_algorithm_params] Algorithm {algo} is not implemented, loading defaults...")
            return None
        block = (self._cfg.get("algorithms") or {}).get(algo)
        if isinstance(block, dict):
            if algo == "REINFORCE":
                params = {k: block[k] for k in REINFORCE_FALLBACK}
            else:
                params = dict(ALGO_FALLBACKS[algo])
                params.update({k: v for k, v in block.items() if not k.startswith("_")})
        else:
            params = dict(ALGO_FALLBACKS[algo])
        return {algo: params}

    @staticmethod
    def _server(sp, port, what) -> Dict[str, str]:
        if _server_ok(sp):
            return {"prefix": sp["prefix"], "host": sp["host"], "port": sp["port"]}
        _log(f"[ConfigLoader] Failed to load {what} configuration, loading defaults...")
        return {"prefix": "tcp://", "host": "*", "port": port}

    def _set_tb_params(self) -> Dict[str, Any]:
        p = (self._cfg.get("tensorboard") or {}).get("training_tensorboard")
        if p is None and _tb_ok(self._cfg.get("training_tensorboard")):
            p = self._cfg["training_tensorboard"]  # default_config.json places it at the top level
        if p is None:
            return {"launch_tb_on_startup": False, "scalar_tags": ["AverageEpRet", "StdEpRet"],
                    "global_step_tag": "Epoch"}
        return {"launch_tb_on_startup": p["launch_tb_on_startup"], "scalar_tags": p["scalar_tags"].split(";"),
                "global_step_tag": p["global_step_tag"]}

    # ------------------------------------------------------------------ getters (Python API)
    def get_algorithm_params(self) -> Optional[Dict[str, Dict[str, Any]]]:
        return copy.deepcopy(self.algorithm_params)

    def get_train_server(self) -> Dict[str, str]:
        return dict(self.train_server)

    def get_traj_server(self) -> Dict[str, str]:
        return dict(self.traj_server)

    def get_agent_listener(self) -> Dict[str, str]:
        return dict(self.agent_listener)

    def get_tb_params(self) -> Dict[str, Any]:
        return {"launch_tb_on_startup": self.tb_params["launch_tb_on_startup"],
                "scalar_tags": list(self.tb_params["scalar_tags"]),
                "global_step_tag": self.tb_params["global_step_tag"]}

    def get_client_model_path(self) -> str:
        return self.client_model_path

    def get_server_model_path(self) -> str:
        return self.server_model_path

    def get_max_traj_length(self) -> int:
        return int(self.max_traj_length)

    def get_grpc_idle_timeout(self) -> int:
        return int(self.grpc_idle_timeout)

    def get_mi355x_params(self) -> Dict[str, Any]:
        return dict(self.mi355x)

    def raw(self) -> Dict[str, Any]:
        return copy.deepcopy(self._cfg)


def address(sp: Dict[str, str], with_prefix: bool = True) -> str:
    """prefix + host + ':' + port (training_server_wrapper.rs:306-327, agent_wrapper.rs:239-251)."""
    host = sp["host"]
    s = f"{host}:{sp['port']}"
    return (sp.get("prefix", "") + s) if with_prefix else s
