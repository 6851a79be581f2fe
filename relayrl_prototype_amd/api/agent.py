"""RelayRLAgent -- Python API of the reference's PyRelayRLAgent (o3_agent.rs:49-329;
agent_wrapper.rs, agent_zmq.rs, agent_grpc.rs).

Per step the agent evaluates its policy locally (CPU numpy MLP from the learner's flat
weights -- no TorchScript interpreter, no per-step safetensors encodes) and appends an
action to the current episode.  Semantics (docs/COMPAT.md):
  * ``request_for_action(obs, mask, reward)``: ``reward`` is the reward of the PREVIOUS
    step (the reference notebooks' calling convention); it is attributed to the previous
    action, fixing the off-by-one alignment of the reference;
  * ``flag_last_action(reward, done=True)`` ends the episode, attaches the final reward to
    the last action and ships the episode (one RRLT frame); ``truncated=True`` ships it
    as a time-limit cut so the learner bootstraps from V(s_T);
  * model updates arrive asynchronously (ZMQ push / gRPC poll after each episode /
    in-process subscription) and are swapped atomically between steps.

``wire_format``: "columns" (one RRLC frame per episode, the default), "actions" (per-action
RRLT frames / protobuf actions), or "reference": the reference agent's own wire, to train
against a reference Rust training server.  ZMQ: GET_MODEL without a format frame,
``serde_pickle(Vec<RelayRLAction>)`` uploads (trajectory.rs:50-90) and TorchScript model
pushes into a PULL this agent binds on ``training_server`` (agent_zmq.rs:316-442, 625-698).
gRPC: ``ClientPoll{first_time: 1}`` handshake, per-episode ``SendActions`` with safetensors
tensor fields, then a synchronous ``ClientPoll{first_time: 0, version}`` that swaps in a
non-empty model (agent_grpc.rs:318-360, 492-599).
Uploads are per episode (the reference re-sent the whole history each time, defect A1); each
action carries its OWN step's reward and ``data = {"logp_a", "v"}`` tensors, and the episode
ends in the reference's terminal marker ``(None, None, None, rew, done=True)`` whose reward is
the REINFORCE.py:86 ``finish_path(last_val)`` bootstrap: 0 after a terminal state, V(s_T)
after a time-limit cut (docs/COMPAT.md).
"""
from __future__ import annotations

import threading
from typing import Optional

import numpy as np

from ..config import ConfigLoader, address, resolve_config_json_path
from ..models.cpu_policy import CPUPolicy
from ..runtime.model_store import ModelBlob
from ..types import EpisodeRecorder, RelayRLAction, RelayRLTrajectory, TrajectoryColumns


class RelayRLAgent:
    def __init__(self, model_path: Optional[str] = None, config_path: Optional[str] = "./config.json",
                 server_type: str = "zmq", training_port: Optional[str] = None,
                 training_prefix: Optional[str] = None, training_host: Optional[str] = None,
                 agent_id: Optional[str] = None, seed: Optional[int] = None, handshake_timeout_s: float = 60.0,
                 wire_format: str = "columns", connection_per_upload: bool = False):
        from ..transport.zmq_transport import make_agent_id

        self.config_path = resolve_config_json_path(config_path)
        self.cfg = ConfigLoader(None, self.config_path)
        self.server_type = (server_type or "zmq").lower()
        self.agent_id = agent_id or make_agent_id()
        ts = dict(self.cfg.get_train_server())
        # NOTE: the reference bound these with port/prefix swapped (o3_agent.rs:89-96, A3)
        if training_prefix is not None:
            ts["prefix"] = training_prefix
        if training_host is not None:
            ts["host"] = training_host
        if training_port is not None:
            ts["port"] = str(training_port)
        self.train_server = ts
        self.max_traj_length = self.cfg.get_max_traj_length()
        self._seed = seed
        self.policy: Optional[CPUPolicy] = None
        self._policy_lock = threading.Lock()
        self.model_path = model_path
        self.enabled = True
        self.transport = None
        self._handshake_timeout = handshake_timeout_s
        if wire_format not in ("columns", "actions", "reference"):
            raise ValueError("wire_format must be 'columns' (RRLC frames), 'actions' (per-action RRLT / protobuf) "
                             "or 'reference' (serde_pickle frames + TorchScript pushes, ZMQ only)")
        if wire_format == "reference" and self.server_type not in ("zmq", "grpc"):
            raise ValueError("wire_format='reference' is the reference's ZMQ / gRPC wire")
        self.wire_format = wire_format
        # reference ZMQ wire only: a new TCP connection per upload, as the reference agent does
        self.connection_per_upload = bool(connection_per_upload)
        self._rec = EpisodeRecorder(self.max_traj_length)
        self._aux = []  # per-action step() dicts of a TorchScript (plugin) policy
        if model_path is not None:
            self._load_model_file(model_path)
        self._connect()
        self.episodes_sent = 0

    # ------------------------------------------------------------------ models
    def _load_model_file(self, path: str):
        """Initial model from a TorchScript file: the built-in MLP layout is recovered as flat
        weights (native policy); any other architecture runs through its ``step``
        (o3_agent.rs:72-80 CModule::load + agent_wrapper.rs validate_model)."""
        import torch

        from ..models.policies import flat_from_module, module_dims

        m = torch.jit.load(path, map_location="cpu")
        try:
            obs_dim, act_dim, hidden, discrete = module_dims(m)
            pi, vf = flat_from_module(m, discrete)
        except Exception:  # noqa: BLE001 -- a plugin's own network
            with open(path, "rb") as f:
                self._set_policy(ModelBlob.from_torchscript(0, f.read()))
            return
        self._set_policy(ModelBlob(0, {"obs_dim": obs_dim, "act_dim": act_dim, "hidden": int(hidden),
                                       "discrete": discrete}, pi.numpy(), None if vf is None else vf.numpy()))

    def _set_policy(self, blob: ModelBlob):
        m = blob.meta
        if blob.is_torchscript:  # validated before it replaces the running policy
            from ..models.ts_policy import TorchScriptPolicy

            pol = TorchScriptPolicy(blob.torchscript())
            pol.version = blob.version
            with self._policy_lock:
                self.policy = pol
            return
        with self._policy_lock:
            if getattr(self.policy, "is_torchscript", False):
                self.policy = None
            if self.policy is None or (self.policy.obs_dim, self.policy.act_dim, self.policy.hidden) != (
                    m["obs_dim"], m["act_dim"], m["hidden"]):
                seed = self._seed if self._seed is not None else (hash(self.agent_id) & 0x7FFFFFFF)
                self.policy = CPUPolicy(m["obs_dim"], m["act_dim"], m["hidden"], m.get("discrete", True), blob.pi,
                                        blob.vf, seed)
            else:
                self.policy.load(blob.pi, blob.vf)
            self.policy.version = blob.version
            self._validate()

    def _validate(self):
        """agent_wrapper.rs:88-168: dims known and a dummy step returns (act, non-empty dict)."""
        p = self.policy
        act, data = p.step(np.zeros(p.obs_dim, np.float32), np.ones(p.act_dim, np.float32))
        if act is None or not data:
            raise RuntimeError("model validation failed")

    @property
    def model_version(self) -> int:
        return -1 if self.policy is None else self.policy.version

    # ------------------------------------------------------------------ transport
    def _connect(self, training_server_address: Optional[str] = None):
        if training_server_address:
            s = training_server_address
            prefix = ""
            if "://" in s:
                prefix, s = s.split("://", 1)
                prefix += "://"
            host, port = s.rsplit(":", 1)
            self.train_server = {"prefix": prefix or self.train_server.get("prefix", ""), "host": host, "port": port}
        if self.server_type == "zmq":
            from ..transport.zmq_transport import ZmqAgentTransport

            al = dict(self.cfg.get_agent_listener())
            tr = dict(self.cfg.get_traj_server())
            for d in (al, tr):
                if d["host"] in ("*", "0.0.0.0"):
                    d["host"] = "127.0.0.1"
            if self.wire_format == "reference":
                from ..transport.zmq_transport import ReferenceZmqAgentTransport

                ts = dict(self.train_server)  # the PULL this agent binds (agent_zmq.rs:625-640)
                self.transport = ReferenceZmqAgentTransport(self.agent_id, address(al), address(tr), address(ts),
                                                            self._set_policy, self._handshake_timeout,
                                                            self.connection_per_upload)
                return
            self.transport = ZmqAgentTransport(self.agent_id, address(al), address(tr), self._set_policy,
                                               self._handshake_timeout)
        elif self.server_type == "grpc":
            from ..transport.grpc_transport import GrpcAgentTransport

            host = self.train_server["host"]
            if host in ("*", "0.0.0.0"):
                host = "127.0.0.1"
            if self.wire_format == "reference":
                from ..transport.grpc_transport import ReferenceGrpcAgentTransport

                self.transport = ReferenceGrpcAgentTransport(f"{host}:{self.train_server['port']}", self._set_policy,
                                                             handshake_timeout_s=self._handshake_timeout)
                return
            self.transport = GrpcAgentTransport(f"{host}:{self.train_server['port']}", self._set_policy,
                                                handshake_timeout_s=self._handshake_timeout)
        elif self.server_type == "local":
            from ..transport.local import LocalAgentTransport

            self.transport = LocalAgentTransport(address(self.train_server), self._set_policy, self.agent_id)
        else:
            raise ValueError(f"server_type must be zmq, grpc or local, not {self.server_type!r}")

    @property
    def _ts_policy(self) -> bool:
        return bool(getattr(self.policy, "is_torchscript", False))

    def _reference_actions(self, cols, vals, done: bool, next_obs=None, aux=None):
        """One episode as the reference agent's actions (agent_zmq.rs:458-571 / agent_grpc.rs:
        372-455): obs / act / mask as f32 tensors (the agent casts all three to Float), the
        step()'s dict as ``data`` -- ``logp_a`` and, with a value head, ``v`` -- then the terminal
        marker ``(None, None, None, rew, done=True)`` (agent_zmq.rs:605-610).  ``vals`` = V(s_t)
        per row (NaN without a value head), recorded next to each row's log-prob in the
        EpisodeRecorder so the two cannot drift apart."""
        acts = []
        grpc = self.server_type == "grpc"
        for i in range(len(cols)):
            if aux is not None:  # a TorchScript policy: its step()'s whole dict (convert_generic_dict)
                data = aux[i]
            else:
                data = {"logp_a": np.array([cols.logp[i]], np.float32)}
                if not np.isnan(vals[i]):
                    data["v"] = np.array([vals[i]], np.float32)
            acts.append(RelayRLAction(np.asarray(cols.obs[i], np.float32), np.asarray(cols.act[i], np.float32),
                                      None if cols.mask is None else np.asarray(cols.mask[i], np.float32),
                                      float(cols.rew[i]), data, False, not grpc))
        acts.append(RelayRLAction(None, None, None, self._reference_last(done, next_obs), None, True,
                                  False))  # agent_zmq.rs:605-610 marker
        return acts

    def _reference_last(self, done: bool, next_obs=None) -> float:
        """The terminal marker's reward: 0 for a finished episode, V(s_T) for a cut one."""
        if done or next_obs is None or self.policy is None:
            return 0.0
        with self._policy_lock:
            v = self.policy.value(np.asarray(next_obs, np.float32).reshape(1, -1))
        return 0.0 if v is None else float(np.asarray(v).reshape(-1)[0])

    def _ship(self, done: bool, next_obs=None):
        if self._ts_policy:
            self._ship_plugin(done, next_obs)
            return
        self._aux.clear()
        if self.wire_format == "reference":
            vals = self._rec.val[:self._rec.n].copy()
            cols = self._rec.take(self.agent_id, self.episodes_sent, done, next_obs)
            if self.server_type == "grpc":
                self.transport.send_actions(self._reference_actions(cols, vals, done, next_obs))  # then ClientPoll
            else:
                # the same bytes as reference_frame(self._reference_actions(...)), written from the
                # columns in C++ (tests/test_reference_agent.py)
                from .. import _native

                act = np.asarray(cols.act, np.float32)  # [n][w] from the recorder
                self.transport.send_trajectory(_native.reference_frame_columns(
                    cols.obs, act, cols.mask, cols.rew, cols.logp, vals, self._reference_last(done, next_obs), True))
            self.episodes_sent += 1
            return
        cols = self._rec.take(self.agent_id, self.episodes_sent, done, next_obs)
        cols.max_length = self.max_traj_length
        if self.server_type == "zmq":
            self.transport.send_trajectory(cols.encode() if self.wire_format == "columns"
                                           else cols.to_trajectory().encode())
        elif self.server_type == "grpc":
            if self.wire_format == "columns":
                self.transport.send_frame(cols.encode())
            else:
                self.transport.send_trajectory_pb(cols.to_trajectory())
        else:
            self.transport.send_trajectory_obj(cols)
        self.episodes_sent += 1

    def _ship_plugin(self, done: bool, next_obs=None):
        """A custom plugin's model is running: the episode goes out in the reference's action
        layout -- each action with its step()'s dict, then the terminal marker whose reward is the
        finish_path bootstrap (agent_zmq.rs:458-610) -- which is what a plugin's
        receive_trajectory iterates over (REINFORCE.py:70-95).  Per-action RRLT frames /
        protobuf actions carry the dicts; RRLC columns could not."""
        vals = self._rec.val[:self._rec.n].copy()
        aux = list(self._aux) if len(self._aux) == self._rec.n else None  # None: the model changed mid-episode
        self._aux.clear()
        cols = self._rec.take(self.agent_id, self.episodes_sent, done, next_obs)
        acts = self._reference_actions(cols, vals, done, next_obs, aux)
        if self.wire_format == "reference":
            if self.server_type == "grpc":
                self.transport.send_actions(acts)
            else:
                from ..transport.serde_pickle import reference_frame

                self.transport.send_trajectory(reference_frame(acts))
        else:
            t = RelayRLTrajectory(self.max_traj_length, None, agent_id=self.agent_id)
            t.seq = self.episodes_sent
            t.actions = acts
            if self.server_type == "zmq":
                self.transport.send_trajectory(t.encode())
            elif self.server_type == "grpc":
                self.transport.send_trajectory_pb(t)
            else:
                self.transport.send_trajectory_obj(t)
        self.episodes_sent += 1

    @property
    def traj(self) -> RelayRLTrajectory:
        """The current (unshipped) episode as reference-style actions (a copy)."""
        r = self._rec
        if r.n == 0:
            return RelayRLTrajectory(self.max_traj_length, None, agent_id=self.agent_id)
        n = r.n
        cols = TrajectoryColumns(r.obs[:n], r.act[:n], r.rew[:n], r.done[:n], None if r.mask is None else r.mask[:n],
                                 r.logp[:n], self.agent_id, self.episodes_sent, self.max_traj_length)
        return cols.to_trajectory()

    def clear_episode(self) -> None:
        self._rec.n = 0
        self._aux.clear()

    # ------------------------------------------------------------------ API
    def request_for_action(self, obs, mask=None, reward: float = 0.0) -> RelayRLAction:
        if not self.enabled:
            raise RuntimeError("agent is disabled")
        if self.policy is None:
            raise RuntimeError("no model loaded")
        rec = self._rec
        rec.set_last_reward(float(reward))
        obs_a = np.asarray(obs, np.float32)
        if rec.full():
            # very long episode: every recorded action now has its reward; ship the segment
            # (not done) with s_T = this observation so the learner bootstraps it with V(s_T)
            self._ship(done=False, next_obs=obs_a)
        with self._policy_lock:
            p = self.policy
            mask_a = np.ones(p.act_dim, np.float32) if mask is None else np.asarray(mask, np.float32)
            nat = getattr(p, "_nat", None)
            if nat is not None and obs_a.size == p.obs_dim and mask_a.size == p.act_dim:
                # the built-in MLP: policy step and the episode row in one native call
                sink = rec.sink(p.obs_dim, p.discrete, p.act_dim)
                obs_a, mask_a = np.ascontiguousarray(obs_a), np.ascontiguousarray(mask_a)
                a0, logp, v = nat.step_row(obs_a, mask_a, sink, rec.n)
                rec.n += 1
                aux = {"logp_a": logp} if v is None else {"logp_a": logp, "v": v}
                return RelayRLAction._trusted(obs_a, a0, mask_a, aux)
            act, data = p.step(obs_a, mask_a)
        if getattr(p, "is_torchscript", False):
            return self._record_plugin_step(obs_a, mask_a, act, data)
        a0 = np.asarray(act[0] if act.ndim >= 1 else act)
        logp = data.get("logp_a")
        v = data.get("v")
        rec.record(obs_a, a0, mask_a, None if logp is None else logp[0],
                   None if v is None else float(np.asarray(v).reshape(-1)[0]))
        aux = {k: np.asarray(v[0], np.float32) for k, v in data.items()}
        action = RelayRLAction(obs_a, a0, mask_a, 0.0, aux, False, False)
        return action

    def _record_plugin_step(self, obs_a, mask_a, act, data) -> RelayRLAction:
        """A TorchScript policy's step, recorded as the reference agent does: the action tensor
        as returned (float32) and the converted dict as the action's data."""
        def first(v):
            a = np.asarray(v, np.float32).reshape(-1)
            return float(a[0]) if a.size else None

        a0 = np.asarray(act, np.float32)
        if a0.ndim > 1 and a0.shape[0] == 1:  # a batched [1, ...] step on a [1, D] observation
            a0 = a0[0]
        logp = data.get("logp_a")
        v = data.get("v")
        self._rec.record(obs_a, a0.reshape(-1), mask_a, None if logp is None else first(logp),
                         None if v is None else first(v))
        self._aux.append(data)
        return RelayRLAction(obs_a, a0, mask_a, 0.0, data, False, False)

    def record_action(self, obs, act, mask=None, reward: float = 0.0, data=None, done: bool = False,
                      reward_update_flag: bool = False) -> RelayRLAction:
        """Record an action the agent's policy did not choose -- a scripted or human controller,
        demonstrations, an exploration override -- as one step of the current episode
        (agent_zmq.rs:585-596 declares this with these arguments and leaves it ``todo!()``).

        ``reward`` is the reward this action received (a later ``request_for_action``, whose
        ``reward`` argument is always the previous step's reward, sets it again); ``done=True``
        ends the episode and uploads it, as ``flag_last_action`` does.  The log-probability stored for the learner is
        ``data["logp_a"]`` when given, else the current policy's log-probability of ``act`` (so an
        on-policy learner's ratios stay defined); ``data["v"]`` likewise, else V(obs) when the
        policy has a value head.  ``reward_update_flag`` is accepted for signature parity (the
        columnar wire carries no per-row flag)."""
        del reward_update_flag
        if not self.enabled:
            raise RuntimeError("agent is disabled")
        if self.policy is None:
            raise RuntimeError("no model loaded")
        rec = self._rec
        obs_a = np.ascontiguousarray(obs, np.float32)
        if rec.full():
            self._ship(done=False, next_obs=obs_a)
        p = self.policy
        mask_a = np.ones(p.act_dim, np.float32) if mask is None else np.ascontiguousarray(mask, np.float32)
        discrete = bool(getattr(p, "discrete", True))
        a0 = np.asarray(act, np.int32).reshape(()) if discrete else np.ascontiguousarray(act, np.float32).reshape(-1)
        data = dict(data or {})
        logp, v = data.get("logp_a"), data.get("v")
        if (logp is None or v is None) and not getattr(p, "is_torchscript", False):
            with self._policy_lock:
                x = obs_a.reshape(1, -1)
                if logp is None:
                    logp = self._log_prob(p, x, mask_a, a0)
                if v is None:
                    vv = p.value(x)
                    v = None if vv is None else float(np.asarray(vv).reshape(-1)[0])
        first = (lambda t: None if t is None else float(np.asarray(t, np.float32).reshape(-1)[0]))
        if getattr(p, "is_torchscript", False):
            self._aux.append(data)
        rec.record(obs_a, a0, mask_a, first(logp), first(v))
        rec.set_last_reward(float(reward))
        aux = {k: np.asarray(x, np.float32) for k, x in data.items() if not isinstance(x, str)}
        if logp is not None:
            aux.setdefault("logp_a", np.asarray(first(logp), np.float32))
        action = RelayRLAction(obs_a, a0, mask_a, float(reward), aux or None, bool(done), False)
        if done:
            self._ship(done=True)
        return action

    @staticmethod
    def _log_prob(p, x, mask_a, a0) -> float:
        """log pi(a0 | x) under the built-in policy (masked log-softmax, or the Gaussian head)."""
        z = np.asarray(p.logits(x, mask_a.reshape(1, -1)), np.float64).reshape(-1)
        if getattr(p, "discrete", True):
            m = z.max()
            return float(z[int(a0)] - m - np.log(np.exp(z - m).sum()))
        ls = np.asarray(p.pi[6], np.float64)
        zz = (np.asarray(a0, np.float64) - z) / np.exp(ls)
        return float((-0.5 * zz * zz - ls - 0.9189385332046727).sum())

    def flag_last_action(self, reward: float = 0.0, done: bool = True, truncated: bool = False,
                         next_obs=None) -> None:
        """Close the episode with the final reward (agent_zmq.rs:605-610).  ``truncated=True``
        marks a time-limit cut: pass the final observation as ``next_obs`` and the learner
        bootstraps the cut path with V(next_obs) (without it, V of the last acted state)."""
        if self._rec.n == 0:
            return
        self._rec.set_last_reward(float(reward))
        cut = truncated or not done
        self._ship(done=not cut, next_obs=next_obs if cut else None)

    def restart_agent(self, training_server_address: Optional[str] = None) -> bool:
        self.disable_agent()
        try:
            self.enable_agent(training_server_address)
            return True
        except Exception as e:
            print(f"[RelayRLAgent] restart failed: {e!r}", flush=True)
            return False

    def disable_agent(self) -> None:
        self.enabled = False
        if self.transport is not None:
            self.transport.close()
            self.transport = None

    def enable_agent(self, training_server_address: Optional[str] = None) -> None:
        if self.transport is None:
            self._connect(training_server_address)
        self.enabled = True

    def close(self):
        self.disable_agent()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
