"""Trajectory-fed algorithms (agents send episodes; the learner batches them).

This is the in-process, GPU-backed replacement of the reference's Python learner
subprocess (python_algorithm_reply.py + REINFORCE.py + replay_buffer.py).  Episodes
arrive as RelayRLTrajectory objects (from the ZMTP / gRPC transports or in-process),
are appended to a flat host staging buffer, and every ``traj_per_epoch`` trajectories
the batch is moved to the GPU once and the whole update runs as HIP kernels:
flat segmented GAE/return scan -> fused policy fwd+bwd -> fused Adam -> value loop.
"""
from __future__ import annotations

import os
import time
from typing import Any, Dict, Optional

import numpy as np
import torch

from ..config import ConfigLoader
from ..ops import FwdMode, mlp_forward, scan_flat
from ..utils.logger import EpochLogger, setup_logger_kwargs
from .base import AlgorithmAbstract
from .learner import PGLearner
from ..types import ReferenceColumns, TrajectoryColumns


class FlatBuffer:
    """Host staging buffer of concatenated paths (replay_buffer.py:18-111 layout)."""

    def __init__(self, obs_dim: int, act_dim: int, size: int, discrete: bool):
        self.obs_dim, self.act_dim, self.size, self.discrete = obs_dim, act_dim, int(size), discrete
        self.obs = np.zeros((self.size, obs_dim), np.float32)
        self.act = np.zeros(self.size, np.int32) if discrete else np.zeros((self.size, act_dim), np.float32)
        self.mask = np.ones((self.size, act_dim), np.float32)
        self.rew = np.zeros(self.size, np.float32)
        self.logp = np.zeros(self.size, np.float32)
        self.has_logp = np.zeros(self.size, bool)
        self.done = np.zeros(self.size, np.float32)
        self.boot = np.zeros(self.size, np.float32)
        # s_T of a cut path (shipped by the agent): its value bootstraps the path end
        self.boot_obs = np.zeros((self.size, obs_dim), np.float32)
        self.has_boot_obs = np.zeros(self.size, bool)
        self.ptr = 0
        self.path_start = 0

    def full(self) -> bool:
        return self.ptr >= self.size

    def store(self, obs, act, mask, rew, logp=None):
        i = self.ptr
        if i >= self.size:
            raise OverflowError("trajectory buffer full (raise buf_size)")
        self.obs[i] = np.asarray(obs, np.float32).reshape(-1)[: self.obs_dim]
        if self.discrete:
            self.act[i] = int(np.asarray(act).reshape(-1)[0]) if act is not None else 0
        else:
            self.act[i] = np.asarray(act, np.float32).reshape(-1)[: self.act_dim]
        self.mask[i] = 1.0 if mask is None else np.asarray(mask, np.float32).reshape(-1)[: self.act_dim]
        self.rew[i] = rew
        if logp is not None:
            self.logp[i] = float(np.asarray(logp).reshape(-1)[0])
            self.has_logp[i] = True
        else:
            self.has_logp[i] = False
        self.done[i] = 0.0
        self.ptr += 1

    def store_block(self, obs, act, mask, rew, logp=None, has_logp=None) -> int:
        """Append up to ``len(rew)`` rows at once (columnar uploads); returns rows stored.
        ``has_logp`` (per row) marks which rows carry a log-prob (reference uploads)."""
        i = self.ptr
        n = min(int(rew.shape[0]), self.size - i)
        if n <= 0:
            return 0
        sl = slice(i, i + n)
        self.obs[sl] = obs[:n].reshape(n, -1)[:, : self.obs_dim]
        if self.discrete:
            self.act[sl] = act[:n].reshape(n, -1)[:, 0]
        else:
            self.act[sl] = act[:n].reshape(n, -1)[:, : self.act_dim]
        self.mask[sl] = 1.0 if mask is None else mask[:n].reshape(n, -1)[:, : self.act_dim]
        self.rew[sl] = rew[:n]
        if logp is not None:
            self.logp[sl] = logp[:n]
        self.has_logp[sl] = (logp is not None) if has_logp is None else has_logp[:n]
        self.done[sl] = 0.0
        self.has_boot_obs[sl] = False
        self.ptr += n
        return n

    def finish_path(self, terminal: bool = True, boot_obs=None, boot_value=None):
        """Close the current path.  A cut (non-terminal) path bootstraps with V(boot_obs) when
        the agent shipped its next observation, with ``boot_value`` when the uploader supplied
        the bootstrap itself (the reference's finish_path(last_val), replay_buffer.py:48-79),
        else with V of its last state (nan marker)."""
        if self.ptr > self.path_start:
            i = self.ptr - 1
            self.done[i] = 1.0
            if boot_value is not None:
                self.boot[i] = float(boot_value)
            else:
                self.boot[i] = np.nan if not terminal else 0.0  # nan = bootstrap with a value
            if not terminal and boot_obs is not None:
                self.boot_obs[i] = np.asarray(boot_obs, np.float32).reshape(-1)[: self.obs_dim]
                self.has_boot_obs[i] = True
        self.path_start = self.ptr

    def take(self, device) -> Dict[str, torch.Tensor]:
        n = self.ptr
        sl = slice(0, n)
        out = {
            "obs": torch.from_numpy(self.obs[sl].copy()),
            "act": torch.from_numpy(self.act[sl].copy()),
            "mask": torch.from_numpy(self.mask[sl].copy()),
            "rew": torch.from_numpy(self.rew[sl].copy()),
            "logp": torch.from_numpy(self.logp[sl].copy()),
            "has_logp": bool(self.has_logp[sl].all()) if n else False,
            # decided on the host, before the copy: the device batch needs no mask buffer
            "mask_trivial": bool((self.mask[sl] == 1).all()) if n else True,
            "done": torch.from_numpy(self.done[sl].copy()),
            "boot": torch.from_numpy(self.boot[sl].copy()),
        }
        idx = np.flatnonzero(self.has_boot_obs[sl])
        out["boot_idx"] = torch.from_numpy(idx.astype(np.int64))
        out["boot_obs"] = torch.from_numpy(self.boot_obs[idx].copy())
        self.has_boot_obs[sl] = False
        self.ptr = 0
        self.path_start = 0
        if torch.device(device).type == "cuda":
            for k, v in out.items():
                if torch.is_tensor(v):
                    out[k] = v.pin_memory().to(device, non_blocking=True)
        return out


class EpisodeIngest:
    """Uploaded trajectories -> FlatBuffer paths with the learner's per-episode semantics.

    Shared by the trajectory learner (REINFORCE.receive_trajectory, REINFORCE.py:70-95) and the
    device engines' agent-upload staging (runtime/engine.py).  Columnar RRLC uploads are split
    at their done flags; per-action uploads (RRLT, protobuf, decoded reference serde_pickle
    frames) follow the reference's terminal-marker convention (an action without obs whose
    reward closes the episode, agent_zmq.rs:605-610).  Finished episodes accumulate in
    ``finished`` as (return, length)."""

    def __init__(self, buffer: FlatBuffer):
        self.buffer = buffer
        self.ep_ret = 0.0
        self.ep_len = 0
        self.steps = 0
        self.finished = []

    def end_episode(self, terminal: bool, boot_value=None):
        self.buffer.finish_path(terminal, boot_value=boot_value)
        self.finished.append((self.ep_ret, self.ep_len))
        self.ep_ret, self.ep_len = 0.0, 0

    def pop_finished(self):
        out, self.finished = self.finished, []
        return out

    def add(self, trajectory) -> None:
        if isinstance(trajectory, TrajectoryColumns):
            self._columns(trajectory)
        elif isinstance(trajectory, ReferenceColumns):
            self._reference_columns(trajectory)
        else:
            self._actions(trajectory)

    def _reference_columns(self, c) -> None:
        """``_actions`` on natively decoded reference rows, a run of action rows at a time: a
        run ends at a terminal marker (no observation) or after a done row."""
        buf = self.buffer
        n = len(c)
        has_obs = c.has_obs.astype(bool)
        done = c.done.astype(bool)
        stops = np.flatnonzero(~has_obs | done)  # markers and done rows end runs
        last_done = None  # done flag of the last stored row (None: nothing stored)
        i = 0
        while i < n:
            if not has_obs[i]:  # reference terminal marker: its reward is the path's bootstrap
                if done[i]:
                    self.ep_ret += float(c.rew[i])
                    self.end_episode(terminal=False, boot_value=float(c.rew[i]))
                i += 1
                continue
            if buf.full():
                break
            k_stop = stops[np.searchsorted(stops, i)] if len(stops) and stops[-1] >= i else n
            j = k_stop + 1 if (k_stop < n and has_obs[k_stop]) else k_stop  # a done row belongs to its run
            seg = slice(i, j)
            act = c.act[seg] if c.act is not None else np.zeros((j - i, 1), np.float32)  # no action: 0
            k = buf.store_block(c.obs[seg], act, None if c.mask is None else c.mask[seg], c.rew[seg], c.logp[seg],
                                has_logp=c.has_logp[seg].astype(bool))
            self.steps += k
            self.ep_ret += float(c.rew[i:i + k].sum())
            self.ep_len += k
            if k:
                last_done = bool(done[i + k - 1])
            if k < j - i:
                break  # buffer full
            if done[j - 1]:
                self.end_episode(terminal=True)
            i = j
        if last_done is False and buf.ptr > buf.path_start:
            buf.finish_path(terminal=False)  # truncated segment: bootstrap from V(s_last)

    def _columns(self, c) -> None:
        buf = self.buffer
        n = len(c)
        ends = np.flatnonzero(c.done[:n]) + 1
        start = 0
        for stop in list(ends) + ([n] if (len(ends) == 0 or ends[-1] != n) else []):
            k = buf.store_block(c.obs[start:stop], c.act[start:stop], None if c.mask is None else c.mask[start:stop],
                                c.rew[start:stop], None if c.logp is None else c.logp[start:stop])
            self.steps += k
            self.ep_ret += float(c.rew[start:start + k].sum())
            self.ep_len += k
            if k < stop - start:  # buffer full: cut the path here
                if buf.ptr > buf.path_start:
                    buf.finish_path(terminal=False)
                return
            if c.done[stop - 1]:
                self.end_episode(terminal=True)
            elif buf.ptr > buf.path_start:
                # cut segment: bootstrap with V(s_T) when the agent shipped s_T, else V(s_last)
                buf.finish_path(terminal=False, boot_obs=getattr(c, "next_obs", None))
            start = stop

    def _actions(self, trajectory) -> None:
        buf = self.buffer
        last = None
        for a in trajectory.get_actions():
            obs = a.get_obs()
            if obs is None:
                # reference-style terminal marker (agent_zmq.rs:605-610): REINFORCE.py:86 calls
                # finish_path(last_val=marker reward), i.e. the reward is the path's bootstrap
                # V(s_T) -- discounted by gamma, 0 after a terminal state -- not a step reward
                if a.get_done():
                    self.ep_ret += a.get_rew()  # REINFORCE.py:75 counts it in EpRet
                    self.end_episode(terminal=False, boot_value=a.get_rew())
                continue
            if buf.full():
                break
            data = a.get_data()
            logp = data.get("logp_a")
            buf.store(obs, a.get_act(), a.get_mask(), a.get_rew(), logp)
            self.steps += 1
            self.ep_ret += a.get_rew()
            self.ep_len += 1
            last = a
            if a.get_done():
                self.end_episode(terminal=True)
        if last is not None and not last.get_done() and buf.ptr > buf.path_start:
            buf.finish_path(terminal=False)  # truncated segment: bootstrap from V(s_last)


class TrajectoryAlgorithm(AlgorithmAbstract):
    ALGO = "reinforce"
    CONFIG_NAME = "REINFORCE"

    def __init__(self, env_dir: str = ".", config_path: Optional[str] = None, obs_dim: int = 4, act_dim: int = 2,
                 buf_size: int = 1000000, device=None, hidden: int = 128, logger_quiet: bool = True, **overrides):
        cfg = ConfigLoader(algorithm_name=self.CONFIG_NAME, config_path=config_path)
        params: Dict[str, Any] = dict(cfg.get_algorithm_params()[self.CONFIG_NAME])
        unknown = []
        for k, v in overrides.items():  # hyperparams override the config (fixes A9)
            if k in params or k in self.EXTRA_KEYS:
                params[k] = bool(v) if isinstance(params.get(k), bool) else v
            else:
                unknown.append(k)
        self.unknown_overrides = unknown
        self.params = params
        self.obs_dim, self.act_dim = int(obs_dim), int(act_dim)
        self.discrete = bool(params.get("discrete", True))
        self.with_baseline = bool(params.get("with_vf_baseline", True))
        self.gamma, self.lam = float(params["gamma"]), float(params["lam"])
        self.traj_per_epoch = int(params["traj_per_epoch"])
        self.seed = int(params["seed"])
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        torch.manual_seed(self.seed)
        np.random.seed(self.seed % (2**32))
        self.save_model_path = cfg.get_server_model_path()
        self.buffer = FlatBuffer(self.obs_dim, self.act_dim, buf_size, self.discrete)
        self._ingest = EpisodeIngest(self.buffer)
        self.learner = self._make_learner(params, hidden)
        exp = self.exp_name()
        self.logger = EpochLogger(**setup_logger_kwargs(exp, self.seed, data_dir=os.path.join(env_dir, "logs")),
                                  quiet=logger_quiet)
        self.logger.save_config({"algorithm": self.CONFIG_NAME, "params": params, "obs_dim": obs_dim,
                                 "act_dim": act_dim, "buf_size": buf_size, "env_dir": env_dir,
                                 "device": str(self.device)})
        self.traj = 0
        self.epoch = 0
        self.version = 0
        self._t_epoch = time.perf_counter()
        self._steps_epoch = 0
        self.last_metrics: Dict[str, Any] = {}

    EXTRA_KEYS = ("hidden",)

    # ------------------------------------------------------------------ hooks
    def exp_name(self) -> str:
        return f"relayrl-{self.ALGO}-info"

    def _make_learner(self, p, hidden) -> PGLearner:
        return PGLearner(self.ALGO, self.obs_dim, self.act_dim, hidden, self.discrete, self.with_baseline,
                         pi_lr=p["pi_lr"], vf_lr=p["vf_lr"], train_vf_iters=p.get("train_vf_iters", 80),
                         train_pi_iters=p.get("train_pi_iters", 1), clip_ratio=p.get("clip_ratio", 0.2),
                         target_kl=p.get("target_kl"), ent_coef=p.get("ent_coef", 0.0), device=self.device,
                         seed=self.seed, use_graphs=False, num_minibatches=p.get("num_minibatches", 1))

    # ------------------------------------------------------------------ API
    def receive_trajectory(self, trajectory) -> bool:
        """REINFORCE.receive_trajectory (REINFORCE.py:70-95) with per-episode semantics."""
        self.traj += 1
        buf = self.buffer
        self._ingest.add(trajectory)
        self._ingested()
        if (self.traj % self.traj_per_epoch == 0) or buf.full():
            self.epoch += 1
            self.train_model()
            self.log_epoch()
            return True
        return False

    def _ingested(self) -> None:
        """Per-episode logger rows and the epoch's step count from the ingest."""
        for ret, ln in self._ingest.pop_finished():
            self.logger.store(EpRet=ret, EpLen=ln)
        self._steps_epoch += self._ingest.steps
        self._ingest.steps = 0

    def train_model(self) -> None:
        d = self.buffer.take(self.device)
        B = d["obs"].shape[0]
        if B == 0:
            return
        H = self.learner.hidden
        obs = d["obs"]
        val = None
        boot = d["boot"]
        if self.learner.vf is not None:
            val = mlp_forward(FwdMode.VALUE, self.learner.vf.params, obs, 1, H)["v"]
            self.logger.store(VVals=val.detach().cpu().numpy())
            # nan boot = cut path: V(s_T) where the agent shipped s_T, else V(last state)
            boot = torch.where(torch.isnan(boot), val, boot)
            bi = d["boot_idx"]
            if bi.numel():
                vb = mlp_forward(FwdMode.VALUE, self.learner.vf.params, d["boot_obs"], 1, H)["v"]
                boot = boot.index_copy(0, bi.to(boot.device), vb.to(boot.dtype))
        else:
            # no value net: nothing to bootstrap with; the reference drops last_val too
            # (replay_buffer.py:74-77)
            boot = torch.zeros_like(boot)
        adv, ret, stats = scan_flat(d["rew"], d["done"], val, boot, self.gamma, self.lam)
        act = d["act"] if self.discrete else None
        actc = None if self.discrete else d["act"]
        logp_old = d["logp"] if d["has_logp"] else None
        if logp_old is None and self.ALGO == "ppo":
            mode = FwdMode.CAT_EVAL if self.discrete else FwdMode.GAUSS_EVAL
            logp_old = mlp_forward(mode, self.learner.pi.params, obs, self.act_dim, H, mask=d["mask"],
                                   act_in=act, actc_in=actc)["logp"]
        self.learner.optimize(obs, act=act, actc=actc, mask=d["mask"], adv=adv, ret=ret, adv_stats=stats,
                              logp_old=logp_old)
        self.version += 1
        self.last_metrics = self.learner.summarize()
        for k in ("LossPi", "DeltaLossPi", "KL", "Entropy", "LossV", "DeltaLossV", "ClipFrac"):
            if k in self.last_metrics:
                self.logger.store(**{k: self.last_metrics[k]})

    def log_epoch(self) -> None:
        dt = max(time.perf_counter() - self._t_epoch, 1e-9)
        lg = self.logger
        lg.log_tabular("Epoch", self.epoch)
        lg.log_tabular("EpRet", with_min_and_max=True)
        lg.log_tabular("EpLen", average_only=True)
        lg.log_tabular("LossPi", average_only=True)
        lg.log_tabular("DeltaLossPi", average_only=True)
        if self.learner.vf is not None:
            lg.log_tabular("VVals", with_min_and_max=True)
            lg.log_tabular("LossV", average_only=True)
            lg.log_tabular("DeltaLossV", average_only=True)
        lg.log_tabular("KL", average_only=True)
        lg.log_tabular("Entropy", average_only=True)
        lg.log_tabular("EnvStepsPerSec", self._steps_epoch / dt)
        lg.log_tabular("LearnerDevice", str(self.device))
        self.last_row = lg.dump_tabular()
        self._t_epoch = time.perf_counter()
        self._steps_epoch = 0

    # ------------------------------------------------------------------ model I/O
    def policy_module(self):
        from ..models.policies import build_policy_module

        vf = self.learner.vf.params if self.learner.vf is not None else None
        return build_policy_module(self.obs_dim, self.act_dim, self.learner.hidden, self.learner.pi.params, vf,
                                   self.discrete)

    def save(self, path: Optional[str] = None) -> None:
        from ..models.policies import export_torchscript

        export_torchscript(self.policy_module(), path or self.save_model_path)

    def model_bytes(self) -> bytes:
        from ..models.policies import torchscript_bytes

        return torchscript_bytes(self.policy_module())

    def get_weights(self) -> Dict[str, Any]:
        w = {"pi": self.learner.pi.params.detach().cpu().clone(), "version": self.version,
             "obs_dim": self.obs_dim, "act_dim": self.act_dim, "hidden": self.learner.hidden,
             "discrete": self.discrete}
        if self.learner.vf is not None:
            w["vf"] = self.learner.vf.params.detach().cpu().clone()
        return w

    def state_dict(self) -> Dict[str, Any]:
        return {"learner": self.learner.state_dict(), "traj": self.traj, "epoch": self.epoch,
                "version": self.version, "params": self.params}

    def load_state_dict(self, sd: Dict[str, Any]):
        self.learner.load_state_dict(sd["learner"])
        self.traj, self.epoch, self.version = int(sd["traj"]), int(sd["epoch"]), int(sd["version"])
