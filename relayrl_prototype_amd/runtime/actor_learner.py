"""Actor-learner decoupling over collectives.

The reference decouples agents and the training server with ZeroMQ / gRPC over TCP:
every trajectory fans in to ONE learner (trajectory.rs:69-90 -> training_zmq.rs:948-1058)
and TorchScript models fan out through files + sockets.  One learner GPU cannot keep up
with many actor GPUs (the learner does ~96 % of the FLOPs of an epoch), so here the
learner is a process GROUP:

  W ranks, one per GPU.  Ranks 0 .. L-1 form the learner group (``learner_ranks`` = L,
  default W).  Every rank acts by default (``learner_acts``); actor a feeds learner
  shard ``a mod L``.  A shard receives its K = actors / L rollouts with point-to-point
  receives straight into ONE contiguous HBM batch (K time-major [T, N] blocks back to
  back, then the K x N final observations -- rollout_learn.py ``blocks``), so every
  actor -> learner transfer is a single message per tensor on its own xGMI link and
  nothing is re-stacked.  The shards then run the fused HIP learner data-parallel:
  one RCCL all-reduce of the flat gradient per optimiser step inside the learner group
  (core.FlatNet.apply), which keeps every learner's weights identical.  Each learner
  sends the new flat weight vector back to its own actors (P2P, again one link each).

Handshake (GET_MODEL / MODEL_SET / ID_LOGGED, agent_zmq.rs:316-442) becomes the
process-group rendezvous + an initial weight broadcast; the agent registry is the rank
table.  Every rollout carries a header: sequence number (heartbeat), episode statistics,
and the version + checksum of the weights it was rolled out with.

``max_lag = 1`` overlaps an actor's rollout of epoch k+1 with the learners' update on
epoch k (IMPALA-style lag-1 pipelining).  Weights arrive in a BACK buffer; the actor
copies back -> front on its compute stream only after the receive completed and only
after the previous rollout kernel was queued, and posts the next receive after that
copy, so a rollout never reads a half-written policy.  Learners send from a snapshot of
the parameters, never from the live vector the next Adam step updates in place.  With
``verify_versions`` the learner checks every received header: version in
[k - max_lag, k] and checksum equal to the one recorded when that version was produced.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from ..algorithms.learner import PGLearner
from ..parallel.comm import Comm, collective_timeout
from ..utils.faults import maybe_stall_at
from ..utils.tracing import PhaseTimer
from .rollout_learn import RolloutLearner

# header (float64): seq, n_episodes, sum_ret, sumsq_ret, max_ret, min_ret, sum_len, version, checksum, wsum
HDR = 10


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
    num_minibatches: int = 1       # PPO only
    clip_ratio: float = 0.2
    target_kl: Optional[float] = None
    ent_coef: float = 0.0
    seed: int = 0
    max_lag: int = 0               # 0 synchronous, 1 = actors roll out on weights one update old
    learner_ranks: int = 0         # L: ranks 0 .. L-1 learn (0 = every rank)
    learner_acts: bool = True      # learner ranks also roll out (colocated actor)
    num_threads: int = 4
    use_graphs: bool = True
    verify_versions: bool = False  # check header version/checksum on the learners (syncs)
    stall_timeout_s: float = 120.0  # per-step watchdog floor (0 = off); budget = max(floor, factor x avg step)
    stall_factor: float = 20.0
    phase_timing: bool = False     # HIP-event phases: Rollout, Gather, Learn, AllReduce, WeightSend, ...

    def to_dict(self):
        return asdict(self)


def weight_checksum(p: torch.Tensor) -> torch.Tensor:
    """(sum, index-weighted sum) in fp64 on the device: a torn or stale weight vector
    changes at least one of them."""
    d = p.detach().double()
    w = torch.arange(1, d.numel() + 1, dtype=torch.float64, device=d.device) / d.numel()
    return torch.stack([d.sum(), (d * w).sum()])


class Topology:
    """Rank roles: who learns, who acts, which learner shard every actor feeds."""

    def __init__(self, world: int, learner_ranks: int, learner_acts: bool):
        L = learner_ranks or world
        if not 1 <= L <= world:
            raise ValueError(f"learner_ranks={learner_ranks} with world_size={world}")
        self.world, self.L = world, L
        self.actors = list(range(world)) if learner_acts else list(range(L, world))
        if not self.actors:
            raise ValueError("no actor ranks: use world_size > learner_ranks or learner_acts=True")
        if len(self.actors) % L:
            raise ValueError(f"{len(self.actors)} actors do not split evenly over {L} learner shards")
        self.K = len(self.actors) // L  # actor blocks per learner shard
        self.learner_acts = learner_acts

    @staticmethod
    def fit_learners(world: int, learner_ranks: int, learner_acts: bool) -> int:
        """The largest learner count <= ``learner_ranks`` whose shards split the actors evenly
        on ``world`` ranks (after an elastic shrink the requested count may no longer fit)."""
        L = min(learner_ranks or world, world)
        while L > 1:
            n_act = world if learner_acts else world - L
            if n_act >= 1 and n_act % L == 0:
                return L
            L -= 1
        return 1

    def learner_of(self, actor: int) -> int:
        return self.actors.index(actor) % self.L

    def shard(self, learner: int) -> List[int]:
        """Actors feeding ``learner``, its own (colocated) actor first."""
        return [a for a in self.actors if self.learner_of(a) == learner]


class _Actor:
    """Rollout engine for one rank: device envs when possible, host C++ envs otherwise."""

    def __init__(self, cfg: ActorLearnerConfig, comm: Comm, device, need_tobs: bool):
        self.device = torch.device(device)
        from .vec_trainer import DEVICE_ENVS

        # device envs (discrete: rollout_kernel; continuous HalfCheetahSynth: the Gaussian
        # rollout_cont_kernel, the reference's ContinuousPolicyNetwork completed, kernel.py:49-75)
        self.kind = "device" if (self.device.type == "cuda" and cfg.env in DEVICE_ENVS) else "host"
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
        self.need_tobs = need_tobs
        self.verify = bool(cfg.verify_versions)
        self.seq = 0
        self.header = torch.zeros(HDR, dtype=torch.float64, device=self.device)

    @property
    def dims(self):
        e = self.eng
        return e.D, e.A, (getattr(e, "continuous", False))

    def rollout(self, version: int):
        """-> (obs_train [T,N,D], obs_last [N,D], act, logp, rew, done, tobs|None, header[HDR])"""
        e = self.eng
        T = e.cfg.rollout_len
        # queued before the rollout: same weights it reads (only checked with verify_versions:
        # otherwise no fp64 reduction per rollout)
        ck = weight_checksum(self.params) if self.verify else None
        if self.kind == "device":
            e.rollout()
            e.epoch += 1
            st = e.ep_stats
            ep = st.sum(0)
            stats = torch.stack([ep[0], ep[1], ep[2], st[:, 3].max(), st[:, 4].min(), ep[5]]).double()
            obs, act, logp, rew, done, tobs = e.obs, e.act, e.logp, e.rew, e.done, e.tobs
        else:
            e.rollout()
            s = {"n": 0.0, "sum": 0.0, "sumsq": 0.0, "max": -1e30, "min": 1e30, "sum_len": 0.0}
            for env in e.envs:
                x = env.take_stats()
                for k in ("n", "sum", "sumsq", "sum_len"):
                    s[k] += x[k]
                if x["n"] > 0:
                    s["max"] = max(s["max"], x["max"])
                    s["min"] = min(s["min"], x["min"])
            stats = torch.tensor([s["n"], s["sum"], s["sumsq"], s["max"], s["min"], s["sum_len"]],
                                 dtype=torch.float64, device=self.device)
            obs, act, logp, rew, done, tobs = e.d_obs, e.d_act, e.d_logp, e.d_rew, e.d_done, e.d_tobs
        self.seq += 1
        h = self.header
        h[0] = float(self.seq)
        h[1:7].copy_(stats)
        h[7] = float(version)
        if ck is not None:
            h[8:10].copy_(ck)
        if self.need_tobs and tobs is None:
            tobs = torch.zeros_like(obs[:T])
        return (obs[:T], obs[T], act, logp, rew, done, tobs if self.need_tobs else None, h)


class ActorLearner:
    def __init__(self, cfg: ActorLearnerConfig, comm: Optional[Comm] = None, device=None, on_stall=None):
        self.cfg = cfg
        self.comm = comm or Comm()
        W = self.comm.world
        if W < 2 and not cfg.learner_acts:
            raise ValueError("actor-learner mode needs world_size >= 2 (learners + actors) "
                             "unless the learners also act (learner_acts=True)")
        if cfg.max_lag not in (0, 1):
            raise ValueError("max_lag must be 0 or 1")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.rank = self.comm.rank
        # comm-phase observability: Rollout / Gather / Learn / WeightSend on the
        # learners, Rollout / SendRollout / WeightRecv on actor-only ranks, and every gradient
        # all-reduce inside the learner group as AllReduce (Comm.timer)
        self.timer = PhaseTimer(self.device, enabled=cfg.phase_timing)
        self.topo = topo = Topology(W, cfg.learner_ranks, cfg.learner_acts)
        self.is_learner = self.rank < topo.L
        self.acts = self.rank in topo.actors
        # the learner group (a collective over the default group: every rank calls new_group)
        if topo.L == W:
            self.lcomm = self.comm
        else:
            grp = dist.new_group(list(range(topo.L)), timeout=collective_timeout()) if W > 1 else None
            self.lcomm = Comm(grp) if self.is_learner else None
        if self.lcomm is not None:
            self.lcomm.timer = self.timer
        need_tobs = cfg.with_baseline or cfg.algo != "reinforce"
        self.actor = _Actor(cfg, self.comm, self.device, need_tobs) if self.acts else None
        if self.actor is not None:
            D, A, cont = self.actor.dims
        else:
            from .. import _native

            e = _native.VecEnv(cfg.env, 1, 0, 1)
            D, A, cont = e.obs_dim, e.act_dim, e.continuous
        self.D, self.A, self.continuous = D, A, cont
        T, N, K = cfg.rollout_len, cfg.num_envs, topo.K
        self.n_actors = len(topo.actors)
        self.version = 0
        self.received = 0
        self.epoch = 0
        self.last_hdr = None
        self._send_works = []
        self._recv_work = None
        self._ck = {}  # version -> checksum (learners, verify_versions)
        if self.is_learner:
            self.learner = PGLearner(cfg.algo, D, A, cfg.hidden, not cont, cfg.with_baseline, cfg.pi_lr, cfg.vf_lr,
                                     cfg.train_vf_iters, cfg.train_pi_iters, cfg.clip_ratio, cfg.target_kl,
                                     cfg.ent_coef, self.device, cfg.seed, self.lcomm, cfg.use_graphs,
                                     num_minibatches=cfg.num_minibatches)
            self.shard = topo.shard(self.rank)
            dev = self.device
            # ONE contiguous shard batch: K [T, N] blocks, then the K x N final observations
            self.b_obs = torch.zeros(K * T * N + K * N, D, device=dev)
            self.b_act = torch.zeros((K, T, N, A) if cont else (K, T, N), dtype=torch.float32 if cont else torch.int32,
                                     device=dev)
            self.b_logp = torch.zeros(K, T, N, device=dev)
            self.b_rew = torch.zeros(K, T, N, device=dev)
            self.b_done = torch.zeros(K, T, N, device=dev)
            self.b_tobs = torch.zeros(K, T, N, D, device=dev) if need_tobs else None
            self.b_hdr = torch.zeros(K, HDR, dtype=torch.float64, device=dev)
            self.rl = RolloutLearner(self.learner, T, N, cfg.gamma, cfg.lam, self.lcomm, self.timer, blocks=K)
            self.wsend = torch.zeros_like(self.learner.pi.params)  # snapshot the P2P sends read
            self.front = self.learner.pi.params
        else:
            self.learner = None
            self.front = self.actor.params
        self.back = torch.zeros_like(self.front) if (self.acts and not self.is_learner) else None
        self._pending_peers = []  # (peer rank, work) of the step's in-flight P2P transfers
        # gloo P2P on device tensors (the one-GPU rehearsal of the multi-rank path) moves the bytes
        # from host threads, outside stream order: the kernels that write a send buffer or still
        # read a receive buffer must have finished before the transfer is posted (RCCL P2P is
        # stream-ordered and needs no fence)
        self._host_p2p = self.device.type == "cuda" and self.comm.backend != "nccl"
        self._seen_seq = {}       # actor rank -> last heartbeat sequence number received
        from ..utils.watchdog import StepWatchdog

        self.watchdog = StepWatchdog(f"rank {self.rank} ({'learner' if self.is_learner else 'actor'})",
                                     cfg.stall_timeout_s if W > 1 else 0.0, cfg.stall_factor, self._diagnose,
                                     on_stall)
        # initial weight broadcast from rank 0 (the handshake's GET_MODEL)
        self.comm.broadcast_(self.front, 0)
        if self.is_learner and self.actor is not None:
            self.actor.params.copy_(self.front)
        if self.is_learner and cfg.verify_versions:
            self._ck[0] = weight_checksum(self.front).cpu()

    # ------------------------------------------------------------------ buffers
    def _slot(self, k: int):
        """Contiguous views of slot k of the shard batch (one P2P message per tensor)."""
        T, N, K = self.cfg.rollout_len, self.cfg.num_envs, self.topo.K
        obs_tr = self.b_obs[k * T * N:(k + 1) * T * N]
        obs_last = self.b_obs[K * T * N + k * N:K * T * N + (k + 1) * N]
        tobs = self.b_tobs[k] if self.b_tobs is not None else None
        return (obs_tr, obs_last, self.b_act[k], self.b_logp[k], self.b_rew[k], self.b_done[k], tobs, self.b_hdr[k])

    # ------------------------------------------------------------------ one step
    def step(self):
        self.watchdog.begin(self.epoch)
        tm = self.timer
        parts = None
        if self.actor is not None:
            with tm.phase("Rollout"):
                parts = self.actor.rollout(self.version_in_use)
        if self.is_learner:
            with tm.phase("Gather"):
                self._gather(parts)
            with tm.phase("Learn"):
                self._learn()
            with tm.phase("WeightSend"):
                self._send_weights()
        else:
            with tm.phase("SendRollout"):
                self._send_rollout(parts)
            with tm.phase("WeightRecv"):
                self._recv_weights()
        self.version += 1
        self.epoch += 1
        self.watchdog.end()

    def _diagnose(self) -> str:
        """What this rank is blocked on (called by the watchdog thread)."""
        waiting = []
        for peer, w in list(self._pending_peers):
            try:
                done = w.is_completed()
            except Exception:
                done = False
            if not done:
                waiting.append(peer)
        waiting = sorted(set(waiting))
        if self.is_learner:
            lost = waiting or [a for a in self.shard if a != self.rank]
            seqs = {a: self._seen_seq.get(a) for a in lost}
            return (f"learner {self.rank} is missing rollout {self.epoch} from actor(s) {lost} "
                    f"(last heartbeat seq {seqs}); the learner group all-reduce may be waiting on a peer shard")
        return (f"actor {self.rank} is waiting on learner {self.topo.learner_of(self.rank)} "
                f"(weights v{self.version + 1 - self.cfg.max_lag})")

    @property
    def version_in_use(self) -> int:
        """Version of the weights the next rollout reads (actors lag by up to max_lag)."""
        if self.is_learner:
            return self.version
        return getattr(self, "_front_version", 0)

    def _gather(self, parts):
        """Fan-in: own rollout -> slot 0 (device copy), remote actors -> their slots (P2P)."""
        maybe_stall_at("gather")
        ops = []
        for k, a in enumerate(self.shard):
            dst = self._slot(k)
            if a == self.rank:
                for d, s in zip(dst, parts):
                    if d is not None:
                        d.copy_(s.reshape(d.shape))
                continue
            for d in dst:
                if d is not None:
                    ops.append(dist.P2POp(dist.irecv, d, a))
        if ops:
            self._p2p_fence()  # the previous learn no longer reads the slots
            works = dist.batch_isend_irecv(ops)
            peers = [op.peer for op in ops] if len(works) == len(ops) else [op.peer for op in ops][:len(works)]
            self._pending_peers = list(zip(peers, works))
            for w in works:
                w.wait()
            self._pending_peers = []

    def _send_rollout(self, parts):
        maybe_stall_at("send")
        dst = self.topo.learner_of(self.rank)
        ops = [dist.P2POp(dist.isend, p.contiguous(), dst) for p in parts if p is not None]
        self._p2p_fence()  # the rollout kernels wrote the parts
        for w in dist.batch_isend_irecv(ops):
            w.wait()  # NCCL: stream order only; the next rollout kernel is queued after the send

    def _send_weights(self):
        remote = [a for a in self.shard if a != self.rank]
        for w in self._send_works:  # the snapshot is free again once its sends completed
            w.wait()
        self._send_works = []
        if self.cfg.verify_versions:
            self._ck[self.version + 1] = weight_checksum(self.learner.pi.params).cpu()
        if self.actor is not None:  # colocated actor: next rollout on the newest weights
            self.actor.params.copy_(self.learner.pi.params)
        if not remote:
            return
        self.wsend.copy_(self.learner.pi.params)
        self._p2p_fence()
        self._send_works = dist.batch_isend_irecv([dist.P2POp(dist.isend, self.wsend, a) for a in remote])

    def _recv_weights(self):
        """Actor: the learner sends v_{k+1} after learning rollout k.  max_lag 0 waits for it;
        max_lag 1 keeps rolling out on v_k and picks v_{k+1} up one step later."""
        src = self.topo.learner_of(self.rank)
        if self._recv_work is not None:  # (lag 1) v_k, posted last step
            self._finish_recv()
        self._p2p_fence()  # front.copy_(back) has read the previous version
        works = dist.batch_isend_irecv([dist.P2POp(dist.irecv, self.back, src)])
        self._recv_work = (self.version + 1, works)
        self._pending_peers = [(src, w) for w in works]
        if self.cfg.max_lag == 0:
            self._finish_recv()

    def _p2p_fence(self):
        if self._host_p2p:
            torch.cuda.current_stream(self.device).synchronize()

    def _finish_recv(self):
        ver, works = self._recv_work
        for w in works:
            w.wait()
        self.front.copy_(self.back)  # compute stream, after the receive and after the last rollout
        self._front_version = ver
        self._recv_work = None

    def finish(self):
        """Drain in-flight weight transfers (every rank then holds the newest weights)."""
        if self._recv_work is not None:
            self._finish_recv()
        for w in self._send_works:
            w.wait()
        self._send_works = []
        self.watchdog.close()

    @property
    def wbuf(self) -> torch.Tensor:
        return self.front

    # ------------------------------------------------------------------ learner
    def _learn(self):
        cfg = self.cfg
        K = self.topo.K
        self.rl.learn(self.b_obs, self.b_act, self.b_rew, self.b_done, self.b_logp, tobs=self.b_tobs)
        self.last_hdr = self.b_hdr
        self.received += K
        self._seen_seq = {a: self.epoch + 1 for a in self.shard}  # headers carry seq = epoch + 1
        if cfg.verify_versions:
            self._verify(self.b_hdr.cpu())

    def _verify(self, hdr):
        k, lag = self.version, self.cfg.max_lag
        for j, a in enumerate(self.shard):
            ver = int(hdr[j, 7].item())
            if not (k - lag <= ver <= k):
                raise RuntimeError(f"actor {a}: rollout {k} used weights v{ver}, allowed v{k - lag}..v{k}")
            ref = self._ck.get(ver)
            if ref is None or not torch.allclose(hdr[j, 8:10], ref, rtol=0, atol=0):
                raise RuntimeError(f"actor {a}: rollout {k} weights do not match v{ver} (torn or stale copy)")
        for v in [v for v in self._ck if v < k - lag]:
            del self._ck[v]

    # ------------------------------------------------------------------ metrics
    @property
    def env_steps(self) -> int:
        """Per-rank share of the job's env steps (x world = total, like the other engines)."""
        return self.epoch * self.cfg.rollout_len * self.cfg.num_envs * self.n_actors // self.comm.world

    def _episode_vec(self):
        """Global (n, sum, sumsq, sum_len, max, min) of the newest rollout, over every actor."""
        dev = "cuda" if self.comm.backend == "nccl" else ("cpu" if self.comm.world > 1 else self.device)
        if self.actor is not None:
            h = self.actor.header.to(dev)
            vec = torch.stack([h[1], h[2], h[3], h[6]])
            mx, mn = h[4:5].clone(), h[5:6].clone()
        else:
            vec = torch.zeros(4, dtype=torch.float64, device=dev)
            mx = torch.full((1,), -1e300, dtype=torch.float64, device=dev)
            mn = torch.full((1,), 1e300, dtype=torch.float64, device=dev)
        self.comm.all_reduce_sum_(vec)
        self.comm.all_reduce_max_(mx)
        self.comm.all_reduce_min_(mn)
        return vec.tolist(), mx.item(), mn.item()

    def episode_sums(self) -> tuple:
        (n, s, _, _), _, _ = self._episode_vec()
        return n, s

    def metrics(self) -> dict:
        """Collective over every rank (episode statistics) and the learner group (losses);
        the episode columns are identical on every rank."""
        import math

        (n, s, sq, sl), mx, mn = self._episode_vec()
        out = {"Epoch": self.epoch, "Version": self.version, "WorldSize": self.comm.world,
               "LearnerRanks": self.topo.L}
        if n > 0:
            mean = s / n
            out.update(AverageEpRet=mean, StdEpRet=math.sqrt(max(sq / n - mean * mean, 0.0)), MaxEpRet=mx,
                       MinEpRet=mn, EpLen=sl / n, Episodes=int(n))
        else:
            nan = float("nan")
            out.update(AverageEpRet=nan, StdEpRet=nan, MaxEpRet=nan, MinEpRet=nan, EpLen=nan, Episodes=0)
        if self.is_learner and self.last_hdr is not None:
            h = self.last_hdr.cpu()
            out["ActorSeqs"] = h[:, 0].tolist()
            out["ActorVersions"] = [int(x) for x in h[:, 7].tolist()]
            out.update(self.learner.summarize())
        out["EnvSteps"] = self.epoch * self.cfg.rollout_len * self.cfg.num_envs * self.n_actors
        if self.timer.enabled:
            out.update(self.timer.columns())
            self.timer.reset()
        return out

    def sync_from_rank0(self, src: int = 0):
        """Make every learner hold learner ``src``'s state and every rank its policy weights
        (after an elastic re-form, parallel/elastic.py, or an auto-resume).  ``src`` must be a
        learner rank (the learner group is ranks 0 .. L-1, so its group rank is ``src``)."""
        if src >= self.topo.L:
            raise ValueError(f"sync source {src} is not a learner rank (L = {self.topo.L})")
        if self.is_learner and self.lcomm is not None and self.lcomm.world > 1:
            self.learner.broadcast_state_(self.lcomm, src)
        self.comm.broadcast_(self.front, src)
        if self.is_learner and self.actor is not None:
            self.actor.params.copy_(self.front)
        vec = torch.tensor([float(self.epoch), float(self.version)], dtype=torch.float64,
                           device="cuda" if self.comm.backend == "nccl" else "cpu")
        self.comm.broadcast_(vec, src)
        self.epoch, self.version = int(vec[0].item()), int(vec[1].item())
        self._front_version = self.version

    # ------------------------------------------------------------------ elastic snapshot
    def snapshot_tensors(self):
        ts = self.learner.state_tensors() if self.learner is not None else []
        if self.learner is None:
            ts.append(self.front)
        return ts

    def counters(self) -> dict:
        return {"epoch": self.epoch, "version": self.version, "received": self.received,
                "_front_version": getattr(self, "_front_version", 0)}

    def set_counters(self, c: dict):
        self.epoch, self.version, self.received = int(c["epoch"]), int(c["version"]), int(c["received"])
        self._front_version = int(c["_front_version"])
        if self.learner is not None and self.actor is not None:
            self.actor.params.copy_(self.learner.pi.params)

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        sd = {"epoch": self.epoch, "version": self.version, "cfg": self.cfg.to_dict()}
        if self.learner is not None:
            sd["learner"] = self.learner.state_dict()
        else:
            sd["front"] = self.front.cpu()
        return sd

    def load_state_dict(self, sd: dict):
        self.epoch, self.version = int(sd["epoch"]), int(sd["version"])
        if self.learner is not None and "learner" in sd:
            self.learner.load_state_dict(sd["learner"])
            if self.actor is not None:
                self.actor.params.copy_(self.learner.pi.params)
        elif "front" in sd:
            self.front.copy_(sd["front"].to(self.device))
            self._front_version = self.version
