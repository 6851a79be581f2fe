"""TrainingServer -- Python API of the reference's PyTrainingServer
(o3_training_server.rs:78-272; training_server_wrapper.rs:235-442).

Differences by design (docs/COMPAT.md):
  * the learner runs in-process on the GPU (HIP kernels) -- no Python subprocess / JSON
    pipe; ``disable_server`` / ``enable_server`` stop and restart the transports while
    the learner keeps its state (the reference respawned the learner and lost it);
  * ``hyperparams`` override the JSON config instead of crashing the algorithm (A9);
  * the ZMQ server pushes model updates over the agent's DEALER connection, so any
    number of agents can attach (A6); ``multiactor`` is accepted for compatibility;
  * ``server_type="local"`` runs agent and learner in one process without sockets;
  * ``engine="vec" | "host" | "actor_learner" | "pixel"`` (or the config's ``"mi355x"``
    block / ``hyperparams={"engine": ...}``) puts a GPU device engine behind the server
    (runtime/engine.py): ``train(...)`` runs it, logs the reference progress.txt columns and
    publishes every update to attached agents; ``world_size > 1`` launches one rank per GPU.
"""
from __future__ import annotations

import os
import threading
import time
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
                 checkpoint_every: int = 0, verbose: bool = False, engine: Optional[str] = None):
        self._t_start = time.perf_counter()  # the time-to-threshold clock starts here
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
        from ..runtime import engine as eng

        ap = (self.cfg.get_algorithm_params() or {}).get(algorithm_name.upper(), {})
        self.engine_spec = eng.resolve_engine(algorithm_name, obs_dim, act_dim, ap, self.cfg.get_mi355x_params(), hp,
                                              engine)
        self.engine = None
        if self.engine_spec is None:
            self.algorithm = make_algorithm(algorithm_name, algorithm_dir, env_dir=env_dir,
                                            config_path=self.config_path, obs_dim=obs_dim, act_dim=act_dim,
                                            buf_size=buf_size, device=device, **hp)
        elif self.engine_spec.world_size > 1:
            self.algorithm = eng.RemoteEngineAlgorithm(self.engine_spec, obs_dim, act_dim,
                                                       os.path.join(env_dir, "engine"), self.cfg.get_server_model_path())
        else:
            self.algorithm = eng.EngineAlgorithm(self.engine_spec, env_dir, self.cfg.get_server_model_path(),
                                                 device=device, agent_buf_size=buf_size)
        self._ckpt = None
        if checkpoint_dir and checkpoint_every > 0:
            from ..utils.checkpoint import periodic_checkpointer

            self._ckpt = periodic_checkpointer(checkpoint_dir, checkpoint_every)
        self.service = LearnerService(self.algorithm, checkpoint_fn=self._ckpt,
                                      model_path=self.cfg.get_server_model_path())
        self.service.start()
        if self.engine_spec is not None:
            if self.engine_spec.world_size > 1:
                self.engine = eng.MultiRankEngineRunner(self.algorithm, self.service, env_dir, self._t_start)
            else:
                self.engine = eng.EngineRunner(self.algorithm, self.service, self._t_start)
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
        if self.engine is None:
            try:
                self.algorithm.save()  # initial server model file, like the first GET_MODEL did
            except Exception as e:  # model export must not take the server down
                if verbose:
                    print(f"[TrainingServer] initial model export failed: {e!r}", flush=True)
        # engine mode: the TorchScript archive is produced lazily (GET_MODEL / close), not on
        # the time-to-threshold clock

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
                self._endpoints.append(ZmqTrainingEndpoint(self.service, al, tr, self.multiactor, self.verbose,
                                                           model_push_addr=address(self.train_server)))
            elif self.server_type == "grpc":
                from ..transport.grpc_transport import GrpcTrainingEndpoint

                addr = f"{self.train_server['host']}:{self.train_server['port']}"
                self._endpoints.append(GrpcTrainingEndpoint(self.service, addr, self.cfg.get_grpc_idle_timeout()))
            else:
                self._local_addr = address(self.train_server)
                local_transport.register(self._local_addr, self.service)
                self._endpoints.append("local")
            self.service.start()
            mi = self.cfg.get_mi355x_params()
            self.service.start_sweeper(float(mi.get("agent_timeout_s", 120.0) or 0.0),
                                       float(mi.get("agent_sweep_period_s", 5.0)))

    def disable_server(self) -> None:
        with self._lock:
            self.service.stop_sweeper()
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
        if self.engine is not None and hasattr(self.engine, "stop"):
            self.engine.stop()
            try:
                self.engine.join(60)
            except Exception as e:  # a failed background run must not block the shutdown
                print(f"[TrainingServer] engine ended with {e!r}", flush=True)
        tr = getattr(self.algorithm, "trainer", None)
        if tr is not None and hasattr(tr, "close"):  # releases the host trainer's CU-masked streams
            tr.close()
        self.disable_server()
        self.service.stop(drain=True)
        if hasattr(self.algorithm, "close"):  # the multi-rank engine's relay sockets
            self.algorithm.close()
        if self.tb is not None:
            self.tb.stop()
        if save:
            try:
                self.algorithm.save()
            except Exception:
                pass

    # ------------------------------------------------------------------ device engine
    def train(self, epochs: Optional[int] = None, target_return: Optional[float] = None, window: int = 100,
              max_seconds: Optional[float] = None, log_every: int = 1, publish_every: int = 1,
              background: bool = False):
        """Run the device engine (see runtime/engine.py) until ``epochs`` epochs, the mean return of
        the newest >= ``window`` episodes reaching ``target_return``, or ``max_seconds``.  Returns a
        TrainResult (``time_to_threshold_s`` is measured from this server's construction);
        ``background=True`` returns at once (``engine.join()`` for the result; ``engine.stop()``
        ends it after the current epoch, on every rank)."""
        if self.engine is None:
            raise RuntimeError("this server learns from agent uploads; construct it with engine=... "
                               "(or an \"engine\" entry in the config's \"mi355x\" block) to train on device envs")
        kw = dict(epochs=epochs, target_return=target_return, window=window, max_seconds=max_seconds,
                  log_every=log_every, publish_every=publish_every)
        if background:  # the agents keep being served meanwhile (both the in-process and the multi-rank engine)
            self.engine.start(**kw)
            return None
        return self.engine.train(**kw)

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
