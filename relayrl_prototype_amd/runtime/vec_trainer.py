"""On-device vectorised actor + learner (the flagship training step).

One epoch on each rank (one process per GPU):

  1. fused rollout kernel: T steps x N envs of policy forward + Philox sampling + env
     physics, written time-major into HBM            (csrc/kernels/rollout.hip)
  2. value forward over the (T+1) x N observations    (mlp_forward VALUE)   [baseline]
  3. GAE / discounted-return scan + adv statistics    (scan.hip)
  4. all-reduce of the 3-float advantage statistics   (RCCL)                 [world > 1]
  5. fused policy fwd+bwd -> slab -> (all-reduce) -> fused Adam              (1 step)
  6. train_vf_iters x fused value fwd+bwd -> Adam, captured as one hipGraph  [baseline]

This is REINFORCE.receive_trajectory + train_model (REINFORCE.py:70-125) restated for a
GPU: the "traj_per_epoch" complete trajectories of the reference become N x T
transitions from N envs, and the per-episode finish_path becomes one scan over the
time-major buffer with done flags.  Data-parallel scaling: every rank runs its own
envs; gradients are summed with one all-reduce per optimiser step (global mean).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Optional

import torch

from ..algorithms.learner import PGLearner
from ..ops import hip
from ..parallel.comm import Comm
from ..utils.tracing import PhaseTimer
from .rollout_learn import RolloutLearner, episode_metrics

DEVICE_ENVS = {"CartPole-v1": 0, "MountainCar-v0": 1, "Acrobot-v1": 2, "LunarLanderSynth-v0": 3,
               "HalfCheetahSynth-v0": 4}
CONTINUOUS_DEVICE_ENVS = {"HalfCheetahSynth-v0"}


class SolvedCheck:
    """Return-threshold test for the time-to-threshold metric: the mean return of the most
    recent >= ``min_episodes`` finished episodes (gymnasium's CartPole-v1 criterion: mean
    >= 475 over 100 consecutive episodes), at epoch granularity -- the newest epochs whose
    episode counts add up to ``min_episodes``.  Feed it VecTrainer.episode_sums() once per
    epoch; it keeps only the epochs the window can still need."""

    def __init__(self, threshold: float = 475.0, min_episodes: int = 100):
        self.threshold = threshold
        self.min_episodes = min_episodes
        self.hist = []  # (n, s) per epoch, oldest first

    def update(self, n: float, s: float) -> float:
        """Add one epoch; returns the window mean (NaN until min_episodes have finished)."""
        self.hist.append((n, s))
        tn = ts = 0.0
        keep = 0
        for en, es in reversed(self.hist):
            tn += en
            ts += es
            keep += 1
            if tn >= self.min_episodes:
                break
        del self.hist[:len(self.hist) - keep]
        return ts / tn if tn >= self.min_episodes else float("nan")

    def solved(self, mean: float) -> bool:
        return mean == mean and mean >= self.threshold


class PendingSums:
    """(episodes, return sum) of one epoch, read when needed: a pinned host slot + the event
    recorded after the copy into it, or an already-known pair."""

    def __init__(self, slot, event=None):
        self.slot, self.event = slot, event

    def result(self) -> tuple:
        if self.event is None:
            return tuple(self.slot)
        self.event.synchronize()
        n, s = self.slot.tolist()
        return n, s


@dataclass
class VecTrainerConfig:
    env: str = "CartPole-v1"
    num_envs: int = 32768          # envs per rank
    rollout_len: int = 64          # T
    hidden: int = 128              # reference: [128, 128] (REINFORCE.py:46,49)
    algo: str = "reinforce"        # reinforce | a2c | ppo
    with_baseline: bool = True
    gamma: float = 0.98            # reference defaults (default_config.json:3-16)
    lam: float = 0.97
    pi_lr: float = 3e-4
    vf_lr: float = 1e-3
    train_vf_iters: int = 80
    train_pi_iters: int = 10       # PPO only
    num_minibatches: int = 1       # PPO only: shuffled minibatches per epoch
    clip_ratio: float = 0.2
    target_kl: Optional[float] = None
    seed: int = 1
    use_graphs: bool = True
    ent_coef: float = 0.0
    max_episode_steps: Optional[int] = None
    phase_timing: bool = False     # per-phase HIP-event timing + roctx ranges

    def to_dict(self):
        return asdict(self)


class VecTrainer:
    def __init__(self, cfg: VecTrainerConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm or Comm()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        assert self.device.type == "cuda", "the vectorised trainer runs the fused HIP rollout kernel"
        if cfg.env not in DEVICE_ENVS:
            raise ValueError(f"no device implementation of env {cfg.env!r}; have {list(DEVICE_ENVS)}")
        self.env_id = DEVICE_ENVS[cfg.env]
        h = hip()
        D, A, NS, max_steps = h.env_dims(self.env_id)
        self.D, self.A, self.NS = D, A, NS
        self.max_steps = cfg.max_episode_steps or max_steps
        N, T, H = cfg.num_envs, cfg.rollout_len, cfg.hidden
        dev = self.device
        rank = self.comm.rank
        # identical initial weights on every rank (seeded), per-rank env RNG streams
        self.continuous = cfg.env in CONTINUOUS_DEVICE_ENVS
        self.learner = PGLearner(cfg.algo, D, A, H, not self.continuous, cfg.with_baseline, cfg.pi_lr, cfg.vf_lr,
                                 cfg.train_vf_iters,
                                 cfg.train_pi_iters, cfg.clip_ratio, cfg.target_kl, cfg.ent_coef, dev, cfg.seed,
                                 self.comm, cfg.use_graphs, num_minibatches=cfg.num_minibatches)
        self.pi, self.vf = self.learner.pi, self.learner.vf
        self.timer = PhaseTimer(dev, enabled=cfg.phase_timing)
        if self.comm.multi and cfg.phase_timing:
            self.comm.timer = self.timer  # AllReduce phase (gradient + statistics all-reduces)
        self.rl = RolloutLearner(self.learner, T, N, cfg.gamma, cfg.lam, self.comm, self.timer)
        self.env_seed = (cfg.seed * 0x9E3779B97F4A7C15 + rank * 0x632BE59BD9B4E019) & 0x7FFFFFFFFFFFFFFF
        # time-major SoA rollout buffers (HBM resident)
        self.obs = torch.zeros(T + 1, N, D, device=dev)
        if self.continuous:
            from .. import _native

            self.act = torch.zeros(T, N, A, device=dev)
            self.env_consts = torch.tensor(_native.env_constants(cfg.env), dtype=torch.float32, device=dev)
        else:
            self.act = torch.zeros(T, N, dtype=torch.int32, device=dev)
        self.logp = torch.zeros(T, N, device=dev)
        self.rew = torch.zeros(T, N, device=dev)
        self.done = torch.zeros(T, N, device=dev)  # 0 running / 1 terminal / 2 time-limit truncation
        # pre-reset observation of truncated steps (read only where done == 2): the scan
        # bootstraps a cut episode with V(s_T) like the reference's last_val
        self.tobs = torch.zeros(T, N, D, device=dev) if cfg.with_baseline or cfg.algo != "reinforce" else None
        self.state = torch.zeros(N, NS, device=dev)
        self.ep_len = torch.zeros(N, dtype=torch.int32, device=dev)
        self.ep_ret = torch.zeros(N, device=dev)
        self.ep_stats = torch.zeros(h.rollout_grid(N), 8, device=dev)
        self.B = T * N
        self.global_B = self.B * self.comm.world
        self.epoch = 0
        self.env_steps = 0  # per rank
        self._first = True

    # ------------------------------------------------------------------ one epoch
    def rollout(self):
        cfg, h = self.cfg, hip()
        step0 = self.epoch * cfg.rollout_len
        if self.continuous:
            h.rollout_cont(self.env_id, self.pi.params, self.env_consts, cfg.hidden, self.state, self.ep_len,
                           self.ep_ret, self.obs, self.act, self.logp, self.rew, self.done, self.tobs, self.ep_stats,
                           self.env_seed, step0, self._first, self.max_steps)
        else:
            h.rollout(self.env_id, self.pi.params, cfg.hidden, self.state, self.ep_len, self.ep_ret, self.obs,
                      self.act, self.logp, self.rew, self.done, self.tobs, self.ep_stats, self.env_seed, step0,
                      self._first, self.max_steps)
        self._first = False

    def train_epoch(self):
        with self.timer.phase("Rollout"):
            self.rollout()
        self.rl.learn(self.obs, self.act, self.rew, self.done, self.logp, tobs=self.tobs)
        self.epoch += 1
        self.env_steps += self.B

    # ------------------------------------------------------------------ metrics
    def metrics(self) -> dict:
        """Synchronising read of the last epoch's statistics (global over ranks)."""
        ep = self.ep_stats.sum(0).tolist()
        mx = self.ep_stats[:, 3].max().item()
        mn = self.ep_stats[:, 4].min().item()
        out = {"Epoch": self.epoch}
        out.update(episode_metrics(self.comm, ep[0], ep[1], ep[2], mx, mn, ep[5]))
        out.update(self.learner.summarize())
        out["EnvSteps"] = self.env_steps * self.comm.world
        out["WorldSize"] = self.comm.world
        if self.timer.enabled:
            out.update(self.timer.columns())
            self.timer.reset()
        return out

    def episode_sums(self) -> tuple:
        """(finished episodes, sum of their returns) in the last epoch, global over ranks,
        from ONE device->host read: the per-epoch check of the time-to-threshold loop.
        metrics() reads every column and the learner's loss slabs (~7 synchronising reads,
        a sizeable share of a 1 ms epoch)."""
        ns = self.ep_stats[:, :2].sum(0)
        if self.comm.multi:
            ns = ns.double()
            if self.comm.backend != "nccl":
                ns = ns.cpu()
            self.comm.all_reduce_sum_(ns)
        n, s = ns.tolist()
        return n, s

    def episode_sums_async(self) -> "PendingSums":
        """episode_sums() without the synchronising read: the two sums are copied into a pinned
        host slot behind the epoch on the stream, and the returned handle's ``result()`` waits
        for that copy only.  The threshold loop (EngineRunner.train) consumes epoch k's handle
        after it has queued epoch k + 1, so the GPU never drains for the check."""
        if self.comm.multi and self.comm.backend != "nccl":
            return PendingSums(self.episode_sums())  # host collective: synchronous anyway
        if not hasattr(self, "_sum_slots"):
            self._sum_slots = [torch.empty(2, dtype=torch.float64, pin_memory=True) for _ in range(3)]
            self._sum_events = [torch.cuda.Event() for _ in range(3)]  # reused: no event per epoch
            self._sum_k = 0
            self._sum_dev = torch.empty(2, dtype=torch.float64, device=self.device)
        ns = self._sum_dev
        hip().column_sums(self.ep_stats, 2, ns)  # one launch (a strided torch sum + cast: ~14 us)
        if self.comm.multi:
            self.comm.all_reduce_sum_(ns)
        slot = self._sum_slots[self._sum_k % 3]  # a handle is consumed before the slot comes round
        ev = self._sum_events[self._sum_k % 3]
        self._sum_k += 1
        slot.copy_(ns, non_blocking=True)
        ev.record()
        return PendingSums(slot, ev)

    def average_ep_return(self) -> float:
        """The value metrics()["AverageEpRet"] would return, from one read."""
        n, s = self.episode_sums()
        return s / n if n > 0 else float("nan")

    def sync_from_rank0(self, src: int = 0):
        """Rank ``src``'s learner state everywhere (after an elastic re-form, parallel/elastic.py,
        or an auto-resume where only some ranks hold the newest checkpoint); each rank keeps
        its own env streams."""
        if self.comm.multi:
            self.learner.broadcast_state_(self.comm, src)

    # elastic epoch-start snapshot (launcher.EpochSnapshot): device tensors + host counters
    def snapshot_tensors(self):
        return self.learner.state_tensors() + [self.state, self.ep_len, self.ep_ret]

    def counters(self) -> dict:
        return {"epoch": self.epoch, "env_steps": self.env_steps, "_first": self._first}

    def set_counters(self, c: dict):
        self.epoch, self.env_steps, self._first = int(c["epoch"]), int(c["env_steps"]), bool(c["_first"])

    def state_dict(self) -> dict:
        return {"learner": self.learner.state_dict(), "epoch": self.epoch, "env_steps": self.env_steps,
                "env_state": self.state.cpu(), "ep_len": self.ep_len.cpu(), "ep_ret": self.ep_ret.cpu(),
                "cfg": self.cfg.to_dict()}

    def load_state_dict(self, sd: dict):
        self.learner.load_state_dict(sd["learner"])
        self.epoch = int(sd["epoch"])
        self.env_steps = int(sd["env_steps"])
        self.state.copy_(sd["env_state"].to(self.device))
        self.ep_len.copy_(sd["ep_len"].to(self.device))
        self.ep_ret.copy_(sd["ep_ret"].to(self.device))
        self._first = False
