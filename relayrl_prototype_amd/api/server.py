"""TrainingServer -- Python API of the reference's PyTrainingServer
(o3_training_server.rs:78-272; training_server_wrapper.rs:235-442).

Differences by design (docs/COMPAT.md):
  * the learner runs in-process on the GPU (HIP kernels) -- no Python subprocess / JSON
    pipe; ``disable_server`` / ``enable_server`` stop and restart the transports while
    the learner keeps its state (the reference respawned the learner and lost it);
  * ``hyperparams`` override the JSON config instead of crashing the algorithm (A9);
  * the ZMQ server pushes model updates over the agent's DEALER connection, so any
    number of agents can attach (A6); ``multiactor`` is accepted for compatibility;
  * ``server_type="local"`` runs agent and learner in one process without sockets.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional, Union

from ..algorithms.registry import make_algorithm, parse_hyperparams
from ..config import ConfigLoader, address, resolve_config_json_path
from ..runtime.learner_service import LearnerService
from ..transport import local as local_transport


class TrainingServer:
    def __init__(self, algorithm_name: str, obs_dim: int, act_dim: int, buf_size: int, tensorboard: bool = False,
                 multiactor: bool = False, env_dir: str = "./env", algorithm_dir: Optional[str] = None,
                 config_path: Optional[str] = "./config.json",
                 hyperparams: Optional[Union[Dict[str, str], List[str]]] = None, server_type: str = "zmq",
                 training_prefix: Optional[str] = None, training_host: Optional[str] = None,
                 training_port: Optional[str] = None, device=None, checkpoint_dir: Optional[str] = None,
                 checkpoint_every: int = 0, verbose: bool = False):
        os.makedirs(env_dir, exist_ok=True)
        self.config_path = resolve_config_json_path(config_path)
        self.cfg = ConfigLoader(algorithm_name, self.config_path)
        self.algorithm_name = algorithm_name
        self.server_type = (server_type or "zmq").lower()
        if self.server_type not in ("zmq", "grpc", "local"):
            raise ValueError(f"server_type must be zmq, grpc or local, not {server_type!r}")
        self.env_dir = env_dir
        self.multiactor = multiactor
        self.verbose = verbose
        hp = parse_hyperparams(hyperparams)
        self.algorithm = make_algorithm(algorithm_name, algorithm_dir, env_dir=env_dir, config_path=self.config_path,
                                        obs_dim=obs_dim, act_dim=act_dim, buf_size=buf_size, device=device, **hp)
        self._ckpt = None
        if checkpoint_dir and checkpoint_every > 0:
            from ..utils.checkpoint import periodic_checkpointer

            self._ckpt = periodic_checkpointer(checkpoint_dir, checkpoint_every)
        self.service = LearnerService(self.algorithm, checkpoint_fn=self._ckpt)
        self.service.start()
        ts = dict(self.cfg.get_train_server())
        if training_prefix is not None:
            ts["prefix"] = training_prefix
        if training_host is not None:
            ts["host"] = training_host
        if training_port is not None:
            ts["port"] = str(training_port)
        self.train_server = ts
        self._endpoints = []
        self._lock = threading.Lock()
        self.tb = None
        if tensorboard:
            from ..utils.tensorboard import ProgressTensorboard

            tb = self.cfg.get_tb_params()
            self.tb = ProgressTensorboard(os.path.join(env_dir, "logs"), tb["scalar_tags"], tb["global_step_tag"])
            self.tb.start()
        self.enable_server()
        try:
            self.algorithm.save()  # initial server model file, like the first GET_MODEL did
        except Exception as e:  # model export must not take the server down
            if verbose:
                print(f"[TrainingServer] initial model export failed: {e!r}", flush=True)

    # ------------------------------------------------------------------ addresses
    def addresses(self) -> List[str]:
        if self.server_type == "grpc":
            return [f"{self.train_server['host']}:{self._grpc_port()}"]
        if self.server_type == "local":
            return [address(self.train_server)]
        al = dict(self.cfg.get_agent_listener())
        tr = dict(self.cfg.get_traj_server())
        return [address(al), address(tr)]

    def _grpc_port(self):
        for e in self._endpoints:
            if hasattr(e, "port"):
                return e.port
        return self.train_server["port"]

    def _zmq_endpoints(self):
        al = dict(self.cfg.get_agent_listener())
        tr = dict(self.cfg.get_traj_server())
        return address(al), address(tr)

    # ------------------------------------------------------------------ lifecycle
    def enable_server(self, training_server_address: Optional[str] = None) -> None:
        with self._lock:
            if self._endpoints:
                return
            if training_server_address:
                self._apply_address(training_server_address)
            if self.server_type == "zmq":
                from ..transport.zmq_transport import ZmqTrainingEndpoint

                al, tr = self._zmq_endpoints()
                self._endpoints.append(ZmqTrainingEndpoint(self.service, al, tr, self.multiactor, self.verbose))
            elif self.server_type == "grpc":
                from ..transport.grpc_transport import GrpcTrainingEndpoint

                addr = f"{self.train_server['host']}:{self.train_server['port']}"
                self._endpoints.append(GrpcTrainingEndpoint(self.service, addr, self.cfg.get_grpc_idle_timeout()))
            else:
                self._local_addr = address(self.train_server)
                local_transport.register(self._local_addr, self.service)
                self._endpoints.append("local")
            self.service.start()

    def disable_server(self) -> None:
        with self._lock:
            for e in self._endpoints:
                if e == "local":
                    local_transport.unregister(self._local_addr, self.service)
                else:
                    e.close()
            self._endpoints = []

    def restart_server(self, training_server_address: Optional[str] = None) -> List[str]:
        self.disable_server()
        self.enable_server(training_server_address)
        return self.addresses()

    def _apply_address(self, addr: str):
        s = addr
        prefix = ""
        if "://" in s:
            prefix, s = s.split("://", 1)
            prefix += "://"
        host, port = s.rsplit(":", 1)
        self.train_server = {"prefix": prefix or self.train_server.get("prefix", ""), "host": host, "port": port}

    def close(self, save: bool = True):
        self.disable_server()
        self.service.stop(drain=True)
        if self.tb is not None:
            self.tb.stop()
        if save:
            try:
                self.algorithm.save()
            except Exception:
                pass

    # ------------------------------------------------------------------ extras
    def wait_idle(self, timeout: float = 60.0) -> bool:
        """Block until every submitted trajectory has been processed."""
        return self.service.join_queue(timeout)

    @property
    def model_version(self) -> int:
        b = self.service.store.latest()
        return -1 if b is None else b.version

    def stats(self) -> dict:
        return {"received": self.service.received, "updates": self.service.updates, "errors": self.service.errors,
                "agents": len(self.service.agents), "dropped_seq": self.service.dropped_seq,
                "version": self.model_version}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
