"""Host-env vectorised trainer: C++ env thread pool on the CPU, policy + learner on the GPU.

Per env step (north star "host-side env stepping feeds the learner
through pinned hipMemcpyAsync overlapped ..."):

   env threads write obs_t into PINNED host memory
   -> H2D copy on a side stream (non_blocking) -> fused sampling kernel (HIP)
   -> D2H actions into pinned memory -> env threads step ...

The envs are split into two halves, each with its own C++ thread pool, stepped
ASYNCHRONOUSLY (``VecEnv.step_async``): while the GPU samples actions for one half, the
other half's threads step, and both pools run at the same time -- every env thread is
busy, not half of them.  The rollout (obs, actions, log-probs) never leaves HBM for the
learner; only rewards / done flags go host -> device once per rollout.  Waiting for a
half's actions is a spin on a non-blocking HIP event (no OS sleep in the loop).

``overlap=True`` (lag-1 pipelining, like the reference's asynchronous agent / trainer
split, training_zmq.rs:549-618): two buffer sets; while the compute stream runs epoch k's
update, a rollout thread steps epoch k+1's envs on a SNAPSHOT of the policy one update
old, on its own HIP streams, into the other buffer set.  Epoch time becomes
max(rollout, learn) instead of their sum.  The learner never reads a buffer before the
rollout that fills it has signalled its event, and the snapshot is copied on the
compute stream after the previous update, so neither side sees a half-written tensor.

On a CPU-only machine the same loop runs with the PyTorch oracle ops (used by the
multi-process gloo tests).
"""
from __future__ import annotations

import threading
import time
from dataclasses import asdict, dataclass
from typing import Optional

import torch

from .. import _native
from ..algorithms.learner import PGLearner
from ..ops import FwdMode, mlp_forward
from ..parallel.comm import Comm
from ..utils.tracing import PhaseTimer
from .rollout_learn import RolloutLearner, episode_metrics


@dataclass
class HostTrainerConfig:
    env: str = "CartPole-v1"
    num_envs: int = 1024           # per rank (split into 2 pipeline halves)
    rollout_len: int = 128
    algo: str = "reinforce"        # reinforce | a2c | ppo
    hidden: int = 128
    with_baseline: bool = True
    gamma: float = 0.99
    lam: float = 0.95
    pi_lr: float = 3e-4
    vf_lr: float = 1e-3
    train_vf_iters: int = 80
    train_pi_iters: int = 10
    num_minibatches: int = 1       # PPO only
    clip_ratio: float = 0.2
    target_kl: Optional[float] = None
    ent_coef: float = 0.0
    seed: int = 0
    num_threads: int = 4
    pipeline: bool = True
    use_graphs: bool = True
    log_std_init: float = -0.5
    phase_timing: bool = False
    overlap: bool = False          # lag-1: roll out epoch k+1 while epoch k's update runs (GPU only)
    native_rollout: bool = True    # GPU: the T-step loop in C++ (csrc/runtime/host_rollout.cpp); False = Python loop
    driver_wait: int = 2           # C++ driver: 0 tight event poll, 1 hipEventSynchronize, 2 poll with back-off
    actor_cus: int = 0             # overlap + native: CUs reserved for the rollout's sampling launches (CU-masked
                                   # streams), the learner's grids sized for the rest.  0 = no partition (measured
                                   # faster on the CartPole / HalfCheetah host presets, docs/PERF_NOTES.md)

    def to_dict(self):
        return asdict(self)


class _Buffers:
    """One rollout's pinned host staging (env side) and HBM buffers (learner side)."""

    def __init__(self, T, N, D, A, continuous, pin, device, with_tobs):
        self.h_obs = torch.zeros(T + 1, N, D, pin_memory=pin)
        self.h_rew = torch.zeros(T, N, pin_memory=pin)
        self.h_done = torch.zeros(T, N, pin_memory=pin)  # 0 / 1 terminal / 2 time-limit truncation
        # pre-reset observations of truncated steps (bootstrap V(s_T) of cut episodes)
        self.h_tobs = torch.zeros(T, N, D, pin_memory=pin) if with_tobs else None
        self.d_tobs = torch.zeros(T, N, D, device=device) if with_tobs else None
        if continuous:
            self.h_act = torch.zeros(T, N, A, pin_memory=pin)
            self.d_act = torch.zeros(T, N, A, device=device)
        else:
            self.h_act = torch.zeros(T, N, dtype=torch.int32, pin_memory=pin)
            self.d_act = torch.zeros(T, N, dtype=torch.int32, device=device)
        self.d_obs = torch.zeros(T + 1, N, D, device=device)
        self.d_logp = torch.zeros(T, N, device=device)
        self.d_rew = torch.zeros(T, N, device=device)
        self.d_done = torch.zeros(T, N, device=device)
        self.ready = torch.cuda.Event() if device.type == "cuda" else None  # rollout landed in HBM


class HostVecTrainer:
    def __init__(self, cfg: HostTrainerConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm or Comm()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        cuda = self.device.type == "cuda"
        N, T = cfg.num_envs, cfg.rollout_len
        halves = 2 if (cfg.pipeline and N >= 2) else 1
        self.halves = halves
        bounds = [0, N // 2, N] if halves == 2 else [0, N]
        self.bounds = bounds
        rank = self.comm.rank
        # GPU + native_rollout: the env pools belong to the HIP extension, whose C++ rollout
        # driver steps them (no Python per step); otherwise the host runtime's pools
        envmod = _native
        self.driver = None
        if cuda and cfg.native_rollout:
            from ..ops import hip

            envmod = hip()
        self.envs = [envmod.VecEnv(cfg.env, bounds[h + 1] - bounds[h], cfg.seed * 1000003 + rank * 7919 + h,
                                   max(1, cfg.num_threads // halves)) for h in range(halves)]
        if envmod is not _native:
            self.driver = envmod.HostRollout(self.envs, bounds)
            self.driver.set_wait_mode(cfg.driver_wait)
        e0 = self.envs[0]
        self.D, self.A, self.continuous = e0.obs_dim, e0.act_dim, e0.continuous
        self.learner = PGLearner(cfg.algo, self.D, self.A, cfg.hidden, not self.continuous, cfg.with_baseline,
                                 cfg.pi_lr, cfg.vf_lr, cfg.train_vf_iters, cfg.train_pi_iters, cfg.clip_ratio,
                                 cfg.target_kl, cfg.ent_coef, self.device, cfg.seed, self.comm, cfg.use_graphs,
                                 cfg.log_std_init, num_minibatches=cfg.num_minibatches)
        self.timer = PhaseTimer(self.device, enabled=cfg.phase_timing)
        if self.comm.multi and cfg.phase_timing:
            self.comm.timer = self.timer
        self.rl = RolloutLearner(self.learner, T, N, cfg.gamma, cfg.lam, self.comm, self.timer)
        self.overlap = bool(cfg.overlap and cuda)
        with_tobs = self.learner.vf is not None
        self.bufs = [_Buffers(T, N, self.D, self.A, self.continuous, cuda, self.device, with_tobs)
                     for _ in range(2 if self.overlap else 1)]
        self.cur = 0  # buffer set of the newest completed rollout
        self.copy_stream = torch.cuda.Stream(self.device) if cuda else None
        self.learn_stream = None
        self._masked = []
        if self.overlap:
            self.actor_stream = torch.cuda.Stream(self.device)
            self.actor_copy_stream = torch.cuda.Stream(self.device)
            self.actor_params = self.learner.pi.params.clone()  # lag-1 snapshot the rollout thread reads
            if self.driver is not None and cfg.actor_cus > 0:
                self._partition_cus(cfg.actor_cus, bounds)
        self._pending = None  # (thread, buffer index) of the rollout running ahead
        self.snapshot_versions = []  # policy version each overlapped rollout acted with
        self._primed = False  # a completed rollout waits in self.bufs[self.cur]
        self._rollout_error = None
        if self.overlap:
            self.learner.before_capture = self._quiesce_rollout
            if self.learner.vloop is not None:
                self.learner.vloop.before_capture = self._quiesce_rollout
        # first observation
        for h, env in enumerate(self.envs):
            env.reset_ptr(self.bufs[0].h_obs[0, bounds[h]].data_ptr())
        self._final_obs = None  # host view of the newest env observation (start of the next rollout)
        self.epoch = 0
        self.env_steps = 0
        self.global_step = 0
        self.timings = {"rollout_s": 0.0, "learn_s": 0.0, "wait_rollout_s": 0.0}

    def _partition_cus(self, n_actor: int, bounds):
        """Split the chip between the overlapped rollout and the learner: the value / policy
        kernels are persistent, one 160 KB-LDS workgroup per CU, so a sampling launch on an
        unpartitioned stream waits for a whole learner kernel to drain (measured: 236 us of
        a 278 us CartPole env step).  The actor gets ``n_actor`` CUs spread over the chip
        through a CU-masked stream, the learner a masked stream over the rest, and every
        grid the learner launches is sized for its share (set_cu_limit)."""
        from ..ops import hip

        h = hip()
        n = h.device_cus()
        n_actor = max(8, min(n_actor, n // 4)) // 8 * 8
        # CU-mask bit i lands on XCC i % 8 (the driver deals mask bits round-robin over the
        # XCCs): bits 0 .. n_actor-1 take n_actor / 8 CUs from every XCD, so the learner's grid
        # (dealt round-robin over the XCDs too) finds the same number of CUs on each.  A
        # stride pick (0, 16, 32, ...) put every actor CU on one XCD and made the learner
        # 1.5x slower there (tools/host_overlap_probe.py).
        actor = list(range(n_actor))
        learner = list(range(n_actor, n))
        a_ptr, l_ptr = h.cu_masked_stream(actor), h.cu_masked_stream(learner)
        self._masked = [a_ptr, l_ptr]
        self.actor_stream = torch.cuda.ExternalStream(a_ptr, device=self.device)
        self.learn_stream = torch.cuda.ExternalStream(l_ptr, device=self.device)
        h.set_cu_limit(len(learner))
        # the learner was built for the whole chip: re-size its gradient slabs for its share
        self.learner._pi_slab = None
        self.learner._opt_graphs.clear()
        if self.learner.vloop is not None:
            self.learner.vloop._key = None
        self.driver = h.HostRollout(self.envs, bounds, len(actor))
        self.driver.set_wait_mode(self.cfg.driver_wait)
        self.cu_split = (len(actor), len(learner))

    def close(self):
        """Release the CU-masked streams and the grid-size limit (overlapped host trainer)."""
        self.finish()
        if self._masked:
            from ..ops import hip

            torch.cuda.synchronize(self.device)
            hip().set_cu_limit(0)
            for p in self._masked:
                hip().destroy_stream(p)
            self._masked = []

    # views of the newest completed rollout (actor_learner.py, tests)
    @property
    def h_obs(self):
        return self.bufs[self.cur].h_obs

    @property
    def h_act(self):
        return self.bufs[self.cur].h_act

    @property
    def d_obs(self):
        return self.bufs[self.cur].d_obs

    @property
    def d_act(self):
        return self.bufs[self.cur].d_act

    @property
    def d_logp(self):
        return self.bufs[self.cur].d_logp

    @property
    def d_rew(self):
        return self.bufs[self.cur].d_rew

    @property
    def d_done(self):
        return self.bufs[self.cur].d_done

    @property
    def d_tobs(self):
        return self.bufs[self.cur].d_tobs

    # ------------------------------------------------------------------ rollout
    @property
    def sample_seed(self) -> int:
        return (self.cfg.seed * 0x9E3779B9 + self.comm.rank * 0x85EBCA6B) & 0x7FFFFFFFFFFF

    def _sample(self, b: _Buffers, params, copy_stream, t, h, step):
        lo, hi = self.bounds[h], self.bounds[h + 1]
        cuda = self.device.type == "cuda"
        mode = FwdMode.GAUSS_SAMPLE if self.continuous else FwdMode.CAT_SAMPLE
        seed = self.sample_seed
        if cuda:
            cs = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(copy_stream):
                b.d_obs[t, lo:hi].copy_(b.h_obs[t, lo:hi], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            cs.wait_event(ev)
            out = {"logp": b.d_logp[t, lo:hi], "act": b.d_act[t, lo:hi]}
            if self.continuous:
                out["mean"] = torch.empty(hi - lo, self.A, device=self.device)
            mlp_forward(mode, params, b.d_obs[t, lo:hi], self.A, self.cfg.hidden, seed=seed, step=step + t,
                        row_offset=lo, out=out)
            b.h_act[t, lo:hi].copy_(b.d_act[t, lo:hi], non_blocking=True)
            done_ev = torch.cuda.Event()  # non-blocking event: synchronize() spins, no OS sleep
            done_ev.record(cs)
            return done_ev
        b.d_obs[t, lo:hi].copy_(b.h_obs[t, lo:hi])
        r = mlp_forward(mode, params, b.d_obs[t, lo:hi], self.A, self.cfg.hidden, seed=seed, step=step + t,
                        row_offset=lo)
        b.d_act[t, lo:hi].copy_(r["act"])
        b.d_logp[t, lo:hi].copy_(r["logp"])
        b.h_act[t, lo:hi].copy_(r["act"])
        return None

    def _step_async(self, b: _Buffers, t, h):
        lo = self.bounds[h]
        self.envs[h].step_async_ptr(b.h_act[t, lo].data_ptr(), b.h_obs[t + 1, lo].data_ptr(),
                                    b.h_rew[t, lo].data_ptr(), b.h_done[t, lo].data_ptr(),
                                    b.h_tobs[t, lo].data_ptr() if b.h_tobs is not None else 0)

    def _rollout_into(self, idx: int, params, copy_stream, step0: int):
        """T env steps into buffer set ``idx`` on the calling thread's current stream."""
        T = self.cfg.rollout_len
        b = self.bufs[idx]
        if self.device.type == "cuda":
            # write-after-read: the previous update (queued on the compute stream, or for the
            # overlapped rollout the ``snap`` event this stream waited on) may still read this
            # buffer set; the copy stream's first H2D into it must wait for that
            copy_stream.wait_stream(torch.cuda.current_stream(self.device))
        if self._final_obs is not None and self._final_obs.data_ptr() != b.h_obs[0].data_ptr():
            b.h_obs[0].copy_(self._final_obs)  # continue every env where the last rollout left it
        if self.driver is not None:
            # C++ loop: one zero-copy sampling launch per half-step on this thread's current
            # stream (ordered after the previous update's reads of these buffers)
            self.driver.run(params, self.cfg.hidden, b.h_obs, b.h_act, b.h_rew, b.h_done, b.h_tobs, b.d_obs,
                            b.d_act, b.d_logp, b.d_rew, b.d_done, b.d_tobs, self.sample_seed, step0)
            b.ready.record(torch.cuda.current_stream(self.device))
            self._final_obs = b.h_obs[T]
            return
        for t in range(T):
            evs = []
            for h in range(self.halves):
                if t > 0:
                    self.envs[h].wait()  # obs_t of half h (its step t-1 ran on the pool)
                evs.append(self._sample(b, params, copy_stream, t, h, step0))
            for h in range(self.halves):
                if evs[h] is not None:
                    evs[h].synchronize()  # actions of half h are on the host; the other half may still sample
                self._step_async(b, t, h)
        for env in self.envs:
            env.wait()
        # last observation + rewards / dones to the device (async on the copy stream)
        if self.device.type == "cuda":
            with torch.cuda.stream(copy_stream):
                b.d_obs[T].copy_(b.h_obs[T], non_blocking=True)
                b.d_rew.copy_(b.h_rew, non_blocking=True)
                b.d_done.copy_(b.h_done, non_blocking=True)
                if b.d_tobs is not None:
                    b.d_tobs.copy_(b.h_tobs, non_blocking=True)
            cs = torch.cuda.current_stream(self.device)
            cs.wait_stream(copy_stream)
            b.ready.record(cs)
        else:
            b.d_obs[T].copy_(b.h_obs[T])
            b.d_rew.copy_(b.h_rew)
            b.d_done.copy_(b.h_done)
            if b.d_tobs is not None:
                b.d_tobs.copy_(b.h_tobs)
        self._final_obs = b.h_obs[T]

    def rollout(self):
        """One synchronous rollout with the current weights into the current buffer set."""
        t0 = time.perf_counter()
        self._rollout_into(self.cur, self.learner.pi.params, self.copy_stream, self.global_step)
        self.global_step += self.cfg.rollout_len
        self.timings["rollout_s"] += time.perf_counter() - t0

    # ------------------------------------------------------------------ epoch
    def train_epoch(self):
        if not self.overlap:
            with self.timer.phase("Rollout"):
                self.rollout()
            t0 = time.perf_counter()
            self._learn(self.cur)
            self.timings["learn_s"] += time.perf_counter() - t0
        else:
            self._train_epoch_overlapped()
        self.epoch += 1
        self.env_steps += self.cfg.num_envs * self.cfg.rollout_len

    def _learn(self, idx: int):
        b = self.bufs[idx]
        if b.ready is not None:
            torch.cuda.current_stream(self.device).wait_event(b.ready)
        self.rl.learn(b.d_obs, b.d_act, b.d_rew, b.d_done, b.d_logp, tobs=b.d_tobs)

    def _launch_ahead(self, idx: int):
        """Roll out into buffer set ``idx`` on a thread, with the weights as of now."""
        ls = self.learn_stream or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(ls):
            self.actor_params.copy_(self.learner.pi.params)  # learner stream, after the previous update
        self.snapshot_versions.append(self.learner.pi.version)
        snap = torch.cuda.Event()
        snap.record(ls)
        step0 = self.global_step
        self.global_step += self.cfg.rollout_len

        def run():
            try:
                torch.cuda.set_device(self.device)
                # this thread's event waits must not invalidate the learner's graph capture
                # (HIP drops every active capture when a default-mode thread synchronises)
                from ..ops import hip

                hip().relax_thread_capture_mode()
                with torch.cuda.stream(self.actor_stream):
                    self.actor_stream.wait_event(snap)
                    t0 = time.perf_counter()
                    self._rollout_into(idx, self.actor_params, self.actor_copy_stream, step0)
                    self.timings["rollout_s"] += time.perf_counter() - t0
            except BaseException as e:  # surfaced on join
                self._rollout_error = e

        th = threading.Thread(target=run, name="relayrl-host-rollout", daemon=True)
        th.start()
        self._pending = (th, idx)

    def _quiesce_rollout(self):
        """Let the rollout running ahead finish before the learner captures a graph (first
        epoch on each buffer set only); ``_join_ahead`` still consumes it afterwards."""
        if self._pending is not None:
            t0 = time.perf_counter()
            self._pending[0].join()
            self.timings["wait_rollout_s"] += time.perf_counter() - t0

    def _join_ahead(self) -> int:
        th, idx = self._pending
        t0 = time.perf_counter()
        th.join()
        self.timings["wait_rollout_s"] += time.perf_counter() - t0
        self._pending = None
        if self._rollout_error is not None:
            e, self._rollout_error = self._rollout_error, None
            raise RuntimeError("host rollout thread failed") from e
        return idx

    def _train_epoch_overlapped(self):
        if not self._primed:  # first epoch: nothing rolled out ahead yet
            self._launch_ahead(self.cur)
            self._join_ahead()
            self._primed = True
        learn_idx = self.cur
        nxt = 1 - learn_idx
        self._launch_ahead(nxt)  # epoch k+1's envs step while epoch k's update runs
        t0 = time.perf_counter()
        if self.learn_stream is not None:
            cs = torch.cuda.current_stream(self.device)
            self.learn_stream.wait_stream(cs)
            with torch.cuda.stream(self.learn_stream):
                with self.timer.phase("Optimize"):
                    self._learn(learn_idx)
            cs.wait_stream(self.learn_stream)  # everything after the epoch sees the update
        else:
            with self.timer.phase("Optimize"):
                self._learn(learn_idx)
        self.timings["learn_s"] += time.perf_counter() - t0
        self.cur = self._join_ahead()

    def finish(self):
        if self._pending is not None:
            self._join_ahead()

    # elastic epoch-start snapshot (launcher.EpochSnapshot): device tensors + host counters
    def snapshot_tensors(self):
        return self.learner.state_tensors()

    def counters(self) -> dict:
        return {"epoch": self.epoch, "env_steps": self.env_steps, "global_step": self.global_step}

    def set_counters(self, c: dict):
        self.finish()
        self.epoch, self.env_steps, self.global_step = int(c["epoch"]), int(c["env_steps"]), int(c["global_step"])
        if self.overlap:
            self.actor_params.copy_(self.learner.pi.params)

    def state_dict(self) -> dict:
        """Learner state + counters.  The C++ env threads' states are not exported: a resumed
        host trainer starts fresh episodes (its env seeds advance with the epoch)."""
        return {"learner": self.learner.state_dict(), "epoch": self.epoch, "env_steps": self.env_steps,
                "global_step": self.global_step, "cfg": self.cfg.to_dict()}

    def load_state_dict(self, sd: dict):
        self.finish()
        self.learner.load_state_dict(sd["learner"])
        self.epoch = int(sd["epoch"])
        self.env_steps = int(sd["env_steps"])
        self.global_step = int(sd.get("global_step", self.epoch * self.cfg.rollout_len))
        if self.overlap:
            self.actor_params.copy_(self.learner.pi.params)

    def sync_from_rank0(self, src: int = 0):
        """Rank ``src``'s learner state everywhere; each rank keeps its own env streams."""
        if self.comm.multi:
            self.learner.broadcast_state_(self.comm, src)
            if self.overlap:
                self.actor_params.copy_(self.learner.pi.params)

    def metrics(self) -> dict:
        tot = {"n": 0.0, "sum": 0.0, "sumsq": 0.0, "max": -1e300, "min": 1e300, "sum_len": 0.0}
        for e in self.envs:
            s = e.take_stats()
            if s["n"] > 0:
                tot["max"] = max(tot["max"], s["max"])
                tot["min"] = min(tot["min"], s["min"])
            for k in ("n", "sum", "sumsq", "sum_len"):
                tot[k] += s[k]
        out = {"Epoch": self.epoch}
        out.update(episode_metrics(self.comm, tot["n"], tot["sum"], tot["sumsq"], tot["max"], tot["min"],
                                   tot["sum_len"]))
        out.update(self.learner.summarize())
        out["EnvSteps"] = self.env_steps * self.comm.world
        out["WorldSize"] = self.comm.world
        out["RolloutS"] = self.timings["rollout_s"]
        out["LearnS"] = self.timings["learn_s"]
        out["WaitRolloutS"] = self.timings["wait_rollout_s"]
        if self.driver is not None:  # per-env-step breakdown of the C++ rollout loop (driver thread)
            st = self.driver.take_stats()
            n = max(st["steps"], 1)
            out.update(HostStepUs=st["total_us"] / n, HostEnvWaitUs=st["env_wait_us"] / n,
                       HostGpuWaitUs=st["gpu_wait_us"] / n, HostLaunchUs=st["launch_us"] / n,
                       HostTailUs=st["tail_us"] / n)
        if self.timer.enabled:
            out.update(self.timer.columns())
            self.timer.reset()
        return out
