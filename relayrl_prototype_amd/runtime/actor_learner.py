"""Actor-learner decoupling over collectives.

The reference decouples agents and the training server with ZeroMQ / gRPC over TCP:
trajectories fan in to one learner (trajectory.rs:69-90 -> training_zmq.rs:948-1058),
TorchScript models fan out through files + sockets.  Here every rank is one process
per GPU:

  rank 0          : learner -- receives every actor's rollout straight into HBM,
                    runs the fused HIP learner, broadcasts the flat weight vector;
  ranks 1 .. W-1  : actors -- fused on-device rollout kernel (or host C++ envs),
                    ship [T, N] SoA rollouts to rank 0 with point-to-point sends
                    (each actor -> learner transfer rides its own xGMI link).

Handshake (GET_MODEL / MODEL_SET / ID_LOGGED, agent_zmq.rs:316-442) becomes the
process-group rendezvous + an initial weight broadcast; the agent registry is the rank
table.  Each rollout carries a header (sequence number, episode statistics) that is the
actor heartbeat; the learner detects stalled actors through the collective timeout.

``max_lag = 1`` overlaps the weight broadcast with the next rollout: actors act with a
policy at most one update old (asynchronous actor-learner, like IMPALA/A3C-style
pipelines); ``max_lag = 0`` is fully synchronous.
"""
from __future__ import annotations

import time
from dataclasses import asdict, dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..algorithms.learner import PGLearner
from ..parallel.comm import Comm
from .rollout_learn import RolloutLearner, episode_metrics

HDR = 8  # header floats: seq, n_episodes, sum_ret, sumsq_ret, max_ret, min_ret, sum_len, version


@dataclass
class ActorLearnerConfig:
    env: str = "CartPole-v1"
    num_envs: int = 4096           # per actor rank
    rollout_len: int = 64
    algo: str = "reinforce"
    hidden: int = 128
    with_baseline: bool = True
    gamma: float = 0.99
    lam: float = 0.95
    pi_lr: float = 3e-4
    vf_lr: float = 1e-3
    train_vf_iters: int = 80
    train_pi_iters: int = 10
    clip_ratio: float = 0.2
    target_kl: Optional[float] = None
    ent_coef: float = 0.0
    seed: int = 0
    max_lag: int = 0
    learner_acts: bool = False     # rank 0 also rolls out (colocated actor)
    num_threads: int = 4
    use_graphs: bool = True

    def to_dict(self):
        return asdict(self)


class _Actor:
    """Rollout engine for one rank: device envs when possible, host C++ envs otherwise."""

    def __init__(self, cfg: ActorLearnerConfig, comm: Comm, device):
        self.device = torch.device(device)
        from .vec_trainer import CONTINUOUS_DEVICE_ENVS, DEVICE_ENVS

        self.kind = "device" if (self.device.type == "cuda" and cfg.env in DEVICE_ENVS
                                 and cfg.env not in CONTINUOUS_DEVICE_ENVS) else "host"
        if self.kind == "device":
            from .vec_trainer import VecTrainer, VecTrainerConfig

            vcfg = VecTrainerConfig(env=cfg.env, num_envs=cfg.num_envs, rollout_len=cfg.rollout_len,
                                    hidden=cfg.hidden, algo=cfg.algo, with_baseline=cfg.with_baseline,
                                    seed=cfg.seed, train_vf_iters=0)
            self.eng = VecTrainer(vcfg, comm, device=self.device)
            self.params = self.eng.pi.params
        else:
            from .host_trainer import HostTrainerConfig, HostVecTrainer

            hcfg = HostTrainerConfig(env=cfg.env, num_envs=cfg.num_envs, rollout_len=cfg.rollout_len,
                                     algo=cfg.algo, hidden=cfg.hidden, with_baseline=cfg.with_baseline,
                                     seed=cfg.seed, num_threads=cfg.num_threads, train_vf_iters=0)
            self.eng = HostVecTrainer(hcfg, comm, device=self.device)
            self.params = self.eng.learner.pi.params
        self.seq = 0

    @property
    def dims(self):
        e = self.eng
        return e.D, e.A, (getattr(e, "continuous", False))

    def rollout(self):
        """-> (obs [T+1,N,D], act, logp, rew, done, header[HDR])"""
        e = self.eng
        if self.kind == "device":
            e.rollout()
            e.epoch += 1
            st = e.ep_stats
            ep = st.sum(0)
            hdr = torch.stack([ep[0], ep[1], ep[2], st[:, 3].max(), st[:, 4].min(), ep[5]])
            out = (e.obs, e.act, e.logp, e.rew, e.done)
        else:
            e.rollout()
            s = {"n": 0.0, "sum": 0.0, "sumsq": 0.0, "max": -1e30, "min": 1e30, "sum_len": 0.0}
            for env in e.envs:
                x = env.take_stats()
                s["n"] += x["n"]
                s["sum"] += x["sum"]
                s["sumsq"] += x["sumsq"]
                s["sum_len"] += x["sum_len"]
                if x["n"] > 0:
                    s["max"] = max(s["max"], x["max"])
                    s["min"] = min(s["min"], x["min"])
            hdr = torch.tensor([s["n"], s["sum"], s["sumsq"], s["max"], s["min"], s["sum_len"]], device=self.device)
            out = (e.d_obs, e.d_act, e.d_logp, e.d_rew, e.d_done)
            e.h_obs[0].copy_(e.h_obs[e.cfg.rollout_len])
        self.seq += 1
        header = torch.cat([torch.tensor([float(self.seq)], device=self.device), hdr.float(),
                            torch.zeros(HDR - 7, device=self.device)])
        return out + (header,)


class ActorLearner:
    def __init__(self, cfg: ActorLearnerConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm or Comm()
        if self.comm.world < 2 and not cfg.learner_acts:
            raise ValueError("actor-learner mode needs world_size >= 2 (rank 0 learns, others act) "
                             "unless the learner also acts (learner_acts=True)")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.rank = self.comm.rank
        self.is_learner = self.rank == 0
        self.actor = _Actor(cfg, self.comm, self.device) if (not self.is_learner or cfg.learner_acts) else None
        # every rank needs the dims; derive them from a throw-away env on the learner
        if self.actor is not None:
            D, A, cont = self.actor.dims
        else:
            from .. import _native

            e = _native.VecEnv(cfg.env, 1, 0, 1)
            D, A, cont = e.obs_dim, e.act_dim, e.continuous
        self.D, self.A, self.continuous = D, A, cont
        T, N = cfg.rollout_len, cfg.num_envs
        self.n_actors = self.comm.world - (0 if cfg.learner_acts else 1)
        self.version = 0
        self.received = 0
        self.epoch = 0
        if self.is_learner:
            # identical init to the actors' policies (same seed)
            self.learner = PGLearner(cfg.algo, D, A, cfg.hidden, not cont, cfg.with_baseline, cfg.pi_lr, cfg.vf_lr,
                                     cfg.train_vf_iters, cfg.train_pi_iters, cfg.clip_ratio, cfg.target_kl,
                                     cfg.ent_coef, self.device, cfg.seed, _SoloComm(),
                                     cfg.use_graphs)
            if self.actor is not None:
                self.actor.params.copy_(self.learner.pi.params)
            W = self.comm.world
            adt = torch.float32 if cont else torch.int32
            ash = (T, N, A) if cont else (T, N)
            self.g_obs = [torch.zeros(T + 1, N, D, device=self.device) for _ in range(W)]
            self.g_act = [torch.zeros(*ash, dtype=adt, device=self.device) for _ in range(W)]
            self.g_logp = [torch.zeros(T, N, device=self.device) for _ in range(W)]
            self.g_rew = [torch.zeros(T, N, device=self.device) for _ in range(W)]
            self.g_done = [torch.zeros(T, N, device=self.device) for _ in range(W)]
            self.g_hdr = [torch.zeros(HDR, device=self.device) for _ in range(W)]
            self.rl = RolloutLearner(self.learner, T, N * self.n_actors, cfg.gamma, cfg.lam, _SoloComm())
            self.wbuf = self.learner.pi.params
        else:
            self.wbuf = self.actor.params
        self._pending = None
        self.last_hdr = None
        # initial weight broadcast (the handshake's GET_MODEL)
        self.comm.broadcast_(self.wbuf, 0)

    # ------------------------------------------------------------------ collectives
    def _exchange_rollout(self, parts):
        """P2P fan-in of the six rollout tensors from every actor to rank 0."""
        names = ("g_obs", "g_act", "g_logp", "g_rew", "g_done", "g_hdr")
        W = self.comm.world
        ops = []
        if self.is_learner:
            for k, name in enumerate(names):
                bufs = getattr(self, name)
                for r in range(W):
                    if r == 0:
                        if self.cfg.learner_acts:
                            bufs[0].copy_(parts[k])
                        continue
                    ops.append(dist.P2POp(dist.irecv, bufs[r], r))
        else:
            for k in range(len(names)):
                ops.append(dist.P2POp(dist.isend, parts[k].contiguous(), 0))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()

    def _bcast_weights(self, async_op: bool):
        if self.comm.world == 1:  # colocated single-GPU actor+learner: weights are shared
            return None
        return dist.broadcast(self.wbuf, src=0, async_op=async_op)

    # ------------------------------------------------------------------ one step
    def step(self):
        cfg = self.cfg
        parts = None
        if self.actor is not None:
            parts = self.actor.rollout()
        if not self.is_learner and cfg.max_lag >= 1 and self._pending is not None:
            pass  # rollout above used the stale params; the new ones land below
        self._exchange_rollout(parts)
        if self.is_learner:
            self._learn()
        if cfg.max_lag >= 1:
            if self._pending is not None:
                self._pending.wait()
            self._pending = self._bcast_weights(async_op=True)  # None on a single rank
        else:
            self._bcast_weights(async_op=False)
        self.version += 1
        self.epoch += 1

    def finish(self):
        if self._pending is not None:
            self._pending.wait()
            self._pending = None

    def _learn(self):
        W = self.comm.world
        ranks = [r for r in range(W) if r != 0 or self.cfg.learner_acts]
        T, N = self.cfg.rollout_len, self.cfg.num_envs
        A = len(ranks)
        cat = lambda bufs: torch.stack([bufs[r] for r in ranks], 1)  # [T(+1), A, N, ...]
        obs = cat(self.g_obs).reshape(T + 1, A * N, self.D)
        act = cat(self.g_act).reshape((T, A * N, self.A) if self.continuous else (T, A * N))
        logp = cat(self.g_logp).reshape(T, A * N)
        rew = cat(self.g_rew).reshape(T, A * N)
        done = cat(self.g_done).reshape(T, A * N)
        self.rl.learn(obs, act, rew, done, logp)
        hdr = torch.stack([self.g_hdr[r] for r in ranks])
        self.last_hdr = hdr
        self.received += A
        if self.actor is not None:
            self.actor.params.copy_(self.learner.pi.params)

    def metrics(self) -> dict:
        if not self.is_learner or self.last_hdr is None:
            return {}
        h = self.last_hdr.double().cpu()
        n, s, sq, mx, mn, sl = h[:, 1].sum().item(), h[:, 2].sum().item(), h[:, 3].sum().item(), \
            h[:, 4].max().item(), h[:, 5].min().item(), h[:, 6].sum().item()
        out = {"Epoch": self.epoch, "Version": self.version, "ActorSeqs": h[:, 0].tolist()}
        out.update(episode_metrics(_SoloComm(), n, s, sq, mx, mn, sl))
        out.update(self.learner.summarize())
        out["EnvSteps"] = self.epoch * self.cfg.rollout_len * self.cfg.num_envs * self.n_actors
        return out


class _SoloComm(Comm):
    """The learner's optimiser runs on one rank: no gradient all-reduce."""

    def __init__(self):
        self.group = None
        self.enabled = False
        self.world = 1
        self.rank = 0
        self.backend = "none"
