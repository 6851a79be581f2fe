"""The GPU engines behind the reference API.

The reference's ``TrainingServer`` always spawns one Python learner that trains on the
trajectories agents upload (o3_training_server.rs:78-151 -> training_server_wrapper.rs:235-380
-> training_zmq.rs / training_grpc.rs).  Here ``TrainingServer(..., engine=...)`` -- or the
config's ``"mi355x": {"engine": ...}`` block, or ``hyperparams={"engine": ...}`` -- puts one of
the device engines behind the same object instead:

  vec            runtime/vec_trainer.py     fused on-device actor + HIP learner per GPU
  host           runtime/host_trainer.py    C++ host env threads + HIP learner
  actor_learner  runtime/actor_learner.py   actor ranks -> learner group over RCCL
  pixel          runtime/pixel_trainer.py   Pong pixels, Nature-CNN A2C

The engine trains on its own vectorised envs; ``TrainingServer.train(...)`` drives epochs,
writes the reference's ``progress.txt`` columns (REINFORCE.py:127-139) through the
EpochLogger and publishes each new policy to the server's ModelStore, so agents attached
over ZMQ / gRPC / local keep receiving models exactly as with the trajectory learner.
With ``world_size > 1`` the ranks run as a ``torch.distributed.run`` CHILD process (one
rank per GPU, RCCL); rank 0 is linked to the API process by an in-memory relay
(engine_relay.py): agent uploads go in and are folded into rank 0's shard, every new policy
comes out and is published to the agents -- no file on the weight path.
"""
from __future__ import annotations

import dataclasses
import json
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import torch

from ..algorithms.base import AlgorithmAbstract

ENGINE_KINDS = ("vec", "host", "actor_learner", "pixel")
# (obs_dim, act_dim) of the built-in envs -> env name (the reference passes only the dims)
ENV_BY_DIMS = {(4, 2): "CartPole-v1", (2, 3): "MountainCar-v0", (6, 3): "Acrobot-v1",
               (8, 4): "LunarLanderSynth-v0", (17, 6): "HalfCheetahSynth-v0"}
# reference hyperparameter name -> trainer config field
_PARAM_MAP = {"gamma": "gamma", "lam": "lam", "pi_lr": "pi_lr", "vf_lr": "vf_lr", "train_vf_iters": "train_vf_iters",
              "train_pi_iters": "train_pi_iters", "clip_ratio": "clip_ratio", "target_kl": "target_kl",
              "ent_coef": "ent_coef", "seed": "seed", "num_minibatches": "num_minibatches", "with_vf_baseline": "with_baseline"}
# "mi355x" block name -> trainer config field
_MI355X_MAP = {"envs_per_actor": "num_envs", "num_envs": "num_envs", "rollout_len": "rollout_len",
               "hidden": "hidden", "use_graphs": "use_graphs", "max_episode_steps": "max_episode_steps",
               "num_threads": "num_threads", "learner_acts": "learner_acts", "max_lag": "max_lag",
               "learner_ranks": "learner_ranks"}


@dataclass
class EngineSpec:
    kind: str
    env: str
    algo: str                     # reinforce | ppo | a2c
    world_size: int = 1
    trainer: Dict[str, Any] = field(default_factory=dict)

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self))

    @staticmethod
    def from_json(s: str) -> "EngineSpec":
        return EngineSpec(**json.loads(s))


def resolve_engine(algorithm_name: str, obs_dim: int, act_dim: int, algo_params: Dict[str, Any],
                   mi355x: Dict[str, Any], hyperparams: Dict[str, Any], engine: Optional[str] = None
                   ) -> Optional[EngineSpec]:
    """EngineSpec from (explicit engine > hyperparams > config "mi355x" block), or None for the
    trajectory learner.  Hyperparameters override the config like everywhere else (A9)."""
    hp = dict(hyperparams or {})
    kind = engine or hp.pop("engine", None) or mi355x.get("engine")
    hp.pop("engine", None)
    if not kind:
        return None
    kind = str(kind).lower()
    if kind not in ENGINE_KINDS:
        raise ValueError(f"engine must be one of {ENGINE_KINDS}, not {kind!r}")
    env = hp.pop("env", None) or mi355x.get("env") or ("PongSynth-v0" if kind == "pixel" else
                                                        ENV_BY_DIMS.get((int(obs_dim), int(act_dim))))
    if env is None:
        raise ValueError(f"no built-in env with obs_dim={obs_dim}, act_dim={act_dim}; name one in the "
                         "'mi355x' config block (\"env\": ...) or hyperparams")
    world = int(hp.pop("world_size", mi355x.get("world_size", 1)) or 1)
    algo = {"REINFORCE": "reinforce", "PPO": "ppo", "A2C": "a2c"}.get(algorithm_name.upper(), "reinforce")
    tr: Dict[str, Any] = {}
    for k, v in (algo_params or {}).items():
        if k in _PARAM_MAP and v is not None:
            tr[_PARAM_MAP[k]] = v
    for k, v in mi355x.items():
        if k in _MI355X_MAP:
            tr[_MI355X_MAP[k]] = v
    for k, v in hp.items():  # explicit overrides win (any trainer field by its own name too)
        tr[_PARAM_MAP.get(k, _MI355X_MAP.get(k, k))] = v
    if kind != "pixel":
        tr["env"] = env
        tr["algo"] = algo
    if kind == "pixel":
        # A2C on pixels: one lr for the shared CNN
        if "pi_lr" in tr and "lr" not in tr:
            tr["lr"] = tr["pi_lr"]
    return EngineSpec(kind, env, algo, world, tr)


def _filter(cls, kw: Dict[str, Any]) -> Dict[str, Any]:
    names = {f.name for f in dataclasses.fields(cls)}
    return {k: v for k, v in kw.items() if k in names}


def make_trainer(spec: EngineSpec, comm=None, device=None):
    kw = dict(spec.trainer)
    if spec.kind == "vec":
        from .vec_trainer import VecTrainer, VecTrainerConfig

        return VecTrainer(VecTrainerConfig(**_filter(VecTrainerConfig, kw)), comm, device)
    if spec.kind == "host":
        from .host_trainer import HostTrainerConfig, HostVecTrainer

        return HostVecTrainer(HostTrainerConfig(**_filter(HostTrainerConfig, kw)), comm, device)
    if spec.kind == "actor_learner":
        from .actor_learner import ActorLearner, ActorLearnerConfig

        return ActorLearner(ActorLearnerConfig(**_filter(ActorLearnerConfig, kw)), comm, device)
    from .pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    return PixelA2CTrainer(PixelA2CConfig(**_filter(PixelA2CConfig, kw)), comm, device)


def _epoch(tr):
    return tr.train_epoch() if hasattr(tr, "train_epoch") else tr.step()


# reference progress.txt columns (REINFORCE.py:127-139, progress.txt:1 of the shipped gRPC run)
_REF_COLS = ("AverageEpRet", "StdEpRet", "MaxEpRet", "MinEpRet", "EpLen", "LossPi", "DeltaLossPi")
_VF_COLS = ("AverageVVals", "StdVVals", "MaxVVals", "MinVVals", "LossV", "DeltaLossV")


class EngineAlgorithm(AlgorithmAbstract):
    """A device engine behind the plugin contract (AlgorithmAbstract, BaseAlgorithm.py:4-39):
    ``train_model`` = one engine epoch, ``log_epoch`` = one reference progress.txt row,
    ``save`` / ``model_bytes`` = the TorchScript policy (kernel.py:87-143 interface)."""

    def __init__(self, spec: EngineSpec, env_dir: str = ".", save_model_path: Optional[str] = None, comm=None,
                 device=None, log: bool = True, agent_buf_size: int = 1 << 20):
        self.spec = spec
        if device is None and torch.cuda.is_available():
            device = torch.device("cuda", torch.cuda.current_device())
        self.trainer = make_trainer(spec, comm, device)
        self.comm = getattr(self.trainer, "comm", None)
        self.rank = 0 if self.comm is None else self.comm.rank
        self.save_model_path = save_model_path or os.path.join(os.getcwd(), "server_model.pt")
        self.version = 0
        self.epoch = 0
        self.ignored_trajectories = 0
        # Agent uploads (the reference's "agents upload -> learner trains on them",
        # training_zmq.rs:994-1031 / REINFORCE.py:70-95): staged on the host as concatenated
        # paths and folded into the NEXT engine epoch's batch as extra rows (their own scan and
        # bootstraps, rollout_learn.RolloutLearner._fold_scan).  For the MLP engines (vec /
        # host); "agent_rows": false in the "mi355x" block / hyperparams turns it off.  With
        # several ranks only rank 0 receives uploads (engine_relay.py) and every rank agrees on
        # the global row count per epoch (RolloutLearner.count_sync).
        lr = self.learner
        self.agent_rows = (bool(spec.trainer.get("agent_rows", True)) and spec.kind in ("vec", "host")
                           and lr is not None and hasattr(self.trainer, "rl"))
        if self.agent_rows:
            # padded device-side batch shape: epochs with uploads replay a captured graph
            self.trainer.rl.agent_rows_enabled = True
            self.trainer.rl.agent_cap = int(spec.trainer.get("agent_rows_cap", agent_buf_size))
        if self.agent_rows and self.comm is not None and self.comm.multi:
            self.trainer.rl.count_sync = True  # fallback (non-capturable learners): host row count
        self.agent_rows_total = 0
        self.agent_episodes = 0
        self.agent_trajectories = 0
        self._agent_returns = []
        if self.agent_rows:
            from ..algorithms.trajectory_algo import EpisodeIngest, FlatBuffer

            self._stage = FlatBuffer(lr.obs_dim, lr.act_dim, int(spec.trainer.get("agent_rows_cap", agent_buf_size)),
                                     lr.discrete)
            self._ingest = EpisodeIngest(self._stage)
            self._stage_lock = threading.Lock()
        self.seed = int(spec.trainer.get("seed", 0))
        self.logger = None
        if log and self.rank == 0:
            from ..utils.logger import EpochLogger, setup_logger_kwargs

            exp = f"relayrl-{spec.algo}-{spec.kind}-info"
            self.logger = EpochLogger(**setup_logger_kwargs(exp, self.seed, data_dir=os.path.join(env_dir, "logs")),
                                      quiet=True)
            self.logger.save_config({"engine": dataclasses.asdict(spec),
                                     "world_size": 1 if self.comm is None else self.comm.world})
        self.last_metrics: Dict[str, Any] = {}

    # ------------------------------------------------------------------ model access
    @property
    def learner(self):
        return getattr(self.trainer, "learner", None)

    @property
    def publishes_policy(self) -> bool:
        """MLP policies can be served to agents (NativePolicy / TorchScript); the CNN cannot."""
        return self.learner is not None and self.spec.kind != "pixel"

    def get_weights(self) -> Dict[str, Any]:
        lr = self.learner
        if lr is None:
            return {"pi": torch.zeros(1), "version": self.version, "obs_dim": 0, "act_dim": 0, "hidden": 0,
                    "discrete": True}
        w = {"pi": lr.pi.params.detach().cpu().clone(), "version": self.version, "obs_dim": lr.obs_dim,
             "act_dim": lr.act_dim, "hidden": lr.hidden, "discrete": lr.discrete}
        if lr.vf is not None:
            w["vf"] = lr.vf.params.detach().cpu().clone()
        return w

    def weights_async(self):
        """get_weights() without draining the stream: the parameters are copied into pinned
        host slots behind the queued work (two slot sets, alternating) and ``result()`` waits
        for that copy only -- rank 0 of a multi-rank engine publishes every epoch this way and
        sends each snapshot one epoch later (run_engine_rank)."""
        lr = self.learner
        if lr is None or lr.pi.params.device.type != "cuda":
            w = self.get_weights()
            return _ReadyWeights(w)
        if not hasattr(self, "_wslots"):
            self._wslots = [{"pi": torch.empty(lr.pi.params.numel(), pin_memory=True),
                             "vf": (torch.empty(lr.vf.params.numel(), pin_memory=True) if lr.vf is not None
                                    else None), "ev": torch.cuda.Event()} for _ in range(2)]
            self._wk = 0
        sl = self._wslots[self._wk % 2]
        self._wk += 1
        sl["ev"].synchronize()  # the copy that last used this slot set (two snapshots ago)
        sl["pi"].copy_(lr.pi.params.detach(), non_blocking=True)
        if sl["vf"] is not None:
            sl["vf"].copy_(lr.vf.params.detach(), non_blocking=True)
        sl["ev"].record()
        meta = {"version": self.version, "obs_dim": lr.obs_dim, "act_dim": lr.act_dim, "hidden": lr.hidden,
                "discrete": lr.discrete, "epoch": self.epoch}
        return _PendingWeights(sl, meta)

    def policy_module(self):
        from ..models.policies import build_policy_module

        lr = self.learner
        if lr is None:
            raise RuntimeError(f"the {self.spec.kind} engine has no MLP policy to export")
        return build_policy_module(lr.obs_dim, lr.act_dim, lr.hidden, lr.pi.params,
                                   None if lr.vf is None else lr.vf.params, lr.discrete)

    def model_bytes(self) -> bytes:
        from ..models.policies import torchscript_bytes

        return torchscript_bytes(self.policy_module())

    def save(self, path: Optional[str] = None) -> None:
        from ..models.policies import export_torchscript

        export_torchscript(self.policy_module(), path or self.save_model_path)

    # ------------------------------------------------------------------ plugin contract
    def receive_trajectory(self, trajectory) -> bool:
        """Stage an agent upload for the next engine epoch (LearnerService worker thread).  The
        engine's own epochs publish the models, so this never reports an update."""
        if not self.agent_rows:
            self.ignored_trajectories += 1  # multi-rank / pixel engines train on their own envs only
            return False
        with self._stage_lock:
            if self._stage.full():
                self.ignored_trajectories += 1  # staging full until the next epoch drains it
                return False
            self._ingest.add(trajectory)
            self.agent_trajectories += 1
        return False

    def _take_agent_rows(self):
        if not self.agent_rows:
            return None
        with self._stage_lock:
            if self._stage.ptr == 0:
                return None
            if self._stage.ptr > self._stage.path_start:  # an open path: close it, bootstrapped
                self._stage.finish_path(terminal=False)
            dev = self.learner.device
            d = self._stage.take(dev)
            fin = self._ingest.pop_finished()
        self.agent_episodes += len(fin)
        self._agent_returns.extend(r for r, _ in fin)
        return d

    def train_model(self) -> None:
        d = self._take_agent_rows()
        if d is not None:
            self.trainer.rl.pending_rows = d
        _epoch(self.trainer)
        if d is not None:
            self.agent_rows_total += int(self.trainer.rl.last_agent_rows)
        self.epoch += 1
        self.version += 1

    def epoch_metrics(self) -> Dict[str, Any]:
        m = self.trainer.metrics() or {}
        if self.agent_rows:
            m["AgentRows"] = int(getattr(self.trainer.rl, "last_agent_rows", 0))
            rets, self._agent_returns = self._agent_returns, []
            m["AgentEpisodes"] = len(rets)
            m["AgentEpRet"] = sum(rets) / len(rets) if rets else float("nan")
        self.last_metrics = m
        return m

    def log_epoch(self, m: Optional[Dict[str, Any]] = None, extra: Optional[Dict[str, float]] = None) -> None:
        if self.logger is None:
            return
        m = self.epoch_metrics() if m is None else m
        lg = self.logger
        nan = float("nan")
        lg.log_tabular("Epoch", self.epoch)
        for k in _REF_COLS:
            lg.log_tabular(k, float(m.get(k, 0.0 if k == "DeltaLossPi" else nan)))
        if self.learner is not None and self.learner.vf is not None:
            vv = {"AverageVVals": m.get("VVals", nan), "LossV": m.get("LossV", nan),
                  "DeltaLossV": m.get("DeltaLossV", nan)}
            for k in _VF_COLS:
                lg.log_tabular(k, float(vv.get(k, nan)))
        lg.log_tabular("KL", float(m.get("KL", nan)))
        lg.log_tabular("Entropy", float(m.get("Entropy", nan)))
        if self.agent_rows:  # uploads folded into this epoch's batch (and their episodes' mean return)
            lg.log_tabular("AgentRows", float(m.get("AgentRows", 0)))
            lg.log_tabular("AgentEpRet", float(m.get("AgentEpRet", nan)))
        for k, v in (extra or {}).items():
            lg.log_tabular(k, float(v))
        lg.dump_tabular()

    def episode_sums(self, m: Optional[Dict[str, Any]] = None):
        """(finished episodes, their return sum) of the last epoch, global over ranks."""
        if m is None and hasattr(self.trainer, "episode_sums"):
            return self.trainer.episode_sums()
        m = self.epoch_metrics() if m is None else m
        n = float(m.get("Episodes", 0) or 0)
        r = m.get("AverageEpRet", float("nan"))
        return n, (n * r if n > 0 and r == r else 0.0)

    def episode_sums_async(self):
        """A handle whose ``result()`` is episode_sums(), read without draining the stream when
        the trainer supports it (VecTrainer.episode_sums_async), else computed now."""
        if hasattr(self.trainer, "episode_sums_async"):
            return self.trainer.episode_sums_async()
        from .vec_trainer import PendingSums

        return PendingSums(self.episode_sums())

    def state_dict(self) -> Dict[str, Any]:
        return {"trainer": self.trainer.state_dict(), "epoch": self.epoch, "version": self.version}

    def load_state_dict(self, sd: Dict[str, Any]):
        self.trainer.load_state_dict(sd["trainer"])
        self.epoch, self.version = int(sd["epoch"]), int(sd["version"])


class _ReadyWeights:
    def __init__(self, w):
        self.w = w

    def result(self) -> Dict[str, Any]:
        return self.w


class _PendingWeights:
    def __init__(self, slot, meta):
        self.slot, self.meta = slot, meta

    def result(self) -> Dict[str, Any]:
        self.slot["ev"].synchronize()
        w = dict(self.meta, pi=self.slot["pi"].clone())
        if self.slot["vf"] is not None:
            w["vf"] = self.slot["vf"].clone()
        return w


@dataclass
class TrainResult:
    epochs: int
    seconds: float
    env_steps: int
    solved: bool
    time_to_threshold_s: Optional[float]   # from TrainingServer construction
    last_window_return: float
    metrics: Dict[str, Any]

    def to_dict(self):
        return dataclasses.asdict(self)


class EngineRunner:
    """Drives an in-process EngineAlgorithm: epochs, the return-threshold check, logging and
    model publishing to the server's LearnerService store."""

    def __init__(self, algo: EngineAlgorithm, service, t_start: float):
        self.algo = algo
        self.service = service
        self.t_start = t_start
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.result: Optional[TrainResult] = None
        self._lock = threading.Lock()
        # ranks whose stop request reaches one rank only (engine_relay STOP -> rank 0) agree on
        # it with one all-reduce per epoch
        self.agree_stop = False

    def _publish(self):
        if self.algo.publishes_policy:
            self.service.updates += 1
            self.service.publish_model()

    def train(self, epochs: Optional[int] = None, target_return: Optional[float] = None, window: int = 100,
              max_seconds: Optional[float] = None, log_every: int = 1, publish_every: int = 1) -> TrainResult:
        """Run until ``epochs`` epochs, the mean return of the newest >= ``window`` finished
        episodes reaching ``target_return`` (checked once per epoch), or ``max_seconds``."""
        from .vec_trainer import SolvedCheck

        if epochs is None and target_return is None and max_seconds is None:
            raise ValueError("give epochs, target_return or max_seconds")
        with self._lock:
            algo = self.algo
            comm = algo.comm
            world = 1 if comm is None else comm.world
            check = SolvedCheck(target_return, window) if target_return is not None else None
            t0 = time.perf_counter()
            e0 = algo.epoch
            steps0 = int(getattr(algo.trainer, "env_steps", 0)) * world
            solved, ttt, win = False, None, float("nan")
            m: Dict[str, Any] = {}
            # without per-epoch logging the threshold check runs one epoch behind: epoch k's
            # episode sums are read after epoch k + 1 is queued, so the GPU never drains for
            # the check (~3 % of a reference-hyperparameter epoch, docs/ROUND4.md); the clock
            # stops when the solved epoch's sums reach the host, as before
            # (only trainers with a non-draining read: the others' sums are synchronous anyway,
            # and the lag would only run one extra epoch past the threshold -- ADVICE r4)
            lag = (check is not None and not log_every and hasattr(algo.trainer, "episode_sums_async")
                   and os.environ.get("RRL_TTT_LAGGED_CHECK", "1") != "0")
            pending = None
            # several ranks: the stop request (STOP reaches rank 0 only) and the wall-clock
            # limit are agreed through a device flag, all-reduced behind each epoch and read one
            # epoch later -- the same decision on every rank at the same epoch, and no stream
            # drain per epoch (the old form was an all-reduce + .item() at the
            # top of every epoch)
            multi = comm is not None and comm.multi
            agree = LaggedFlag(comm) if (multi and (self.agree_stop or max_seconds is not None)) else None
            while True:
                if agree is None and self._stop.is_set():
                    break
                algo.train_model()
                k = algo.epoch - e0
                # every rank takes the same branches: metrics() / episode_sums() are collectives
                log_now = bool(log_every) and k % log_every == 0
                m = algo.epoch_metrics() if log_now else {}
                if check is not None and lag:
                    nxt = algo.episode_sums_async()
                    if pending is not None:
                        win = check.update(*pending.result())
                        if check.solved(win):
                            solved = True
                            ttt = time.perf_counter() - self.t_start
                    pending = nxt
                elif check is not None:
                    win = check.update(*algo.episode_sums(m if log_now else None))
                    if check.solved(win):
                        solved = True
                        ttt = time.perf_counter() - self.t_start
                if log_now:
                    el = time.perf_counter() - t0
                    extra = {"Time": el}
                    if "EnvSteps" in m and el > 0:
                        extra["EnvStepsPerSec"] = (m["EnvSteps"] - steps0) / el
                    # the threshold metric as progress columns, on every row (the
                    # table's columns are fixed by its first row): the mean return of the newest
                    # >= window episodes, and the TTT once it is reached (NaN before / unchecked)
                    extra["WindowRet"] = win
                    extra["TimeToThreshold"] = ttt if solved else float("nan")
                    algo.log_epoch(m, extra)
                if publish_every and k % publish_every == 0:
                    self._publish()
                if solved:
                    break
                if epochs is not None and k >= epochs:
                    break
                if agree is not None:
                    timeout = max_seconds is not None and time.perf_counter() - t0 >= max_seconds
                    if agree.post(self._stop.is_set() or timeout):
                        break
                elif max_seconds is not None and time.perf_counter() - t0 >= max_seconds:
                    break
            if pending is not None and not solved:  # the last epoch's sums, still unread
                win = check.update(*pending.result())
                if check.solved(win):
                    solved = True
                    ttt = time.perf_counter() - self.t_start
            if not publish_every or (algo.epoch - e0) % publish_every:
                self._publish()
            el = time.perf_counter() - t0
            steps = int(getattr(algo.trainer, "env_steps", 0)) * world - steps0
            self.result = TrainResult(algo.epoch - e0, el, steps, solved, ttt, win,
                                      {k: v for k, v in m.items() if isinstance(v, (int, float))})
            return self.result

    def start(self, **kw):
        """Train in a background thread (``join()`` for the result)."""
        self._stop.clear()
        self._thread = threading.Thread(target=lambda: self.train(**kw), name="relayrl-engine", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()

    def join(self, timeout: Optional[float] = None) -> Optional[TrainResult]:
        if self._thread is not None:
            self._thread.join(timeout)
        return self.result


class LaggedFlag:
    """A boolean the ranks agree on (true on every rank if it was true on any), decided one
    epoch late without draining the stream: ``post(flag)`` writes this epoch's local flag into
    a device scalar, all-reduces it (MAX) on the stream behind the epoch and copies the result
    into a pinned slot with an event; it returns the agreed flag of the PREVIOUS post, waiting
    only for that older event (the epoch just queued keeps the GPU busy meanwhile).  Every
    rank posts once per epoch, so every rank sees the same sequence of agreed values.  A gloo
    group all-reduces on the host (synchronous, nothing to overlap)."""

    def __init__(self, comm):
        self.comm = comm
        self.on_dev = comm.backend == "nccl" and torch.cuda.is_available()
        dev = torch.device("cuda", torch.cuda.current_device()) if self.on_dev else torch.device("cpu")
        self.flag = torch.zeros(1, device=dev)
        self.slots = [torch.zeros(1, pin_memory=self.on_dev) for _ in range(2)]
        self.events = [torch.cuda.Event() for _ in range(2)] if self.on_dev else None
        self.k = 0
        self.posts = 0

    def post(self, flag: bool) -> bool:
        self.flag.fill_(1.0 if flag else 0.0)
        self.comm.all_reduce_max_(self.flag)
        i = self.k % 2
        self.k += 1
        self.posts += 1
        if not self.on_dev:
            return bool(self.flag[0] > 0)
        self.slots[i].copy_(self.flag, non_blocking=True)
        self.events[i].record()
        if self.k == 1:
            return False
        j = 1 - i
        self.events[j].synchronize()
        return bool(self.slots[j][0] > 0)


# ---------------------------------------------------------------------- multi-rank (child ranks)
class RemoteEngineAlgorithm(AlgorithmAbstract):
    """API-side view of an engine whose ranks run in a child ``torch.distributed.run``.

    Holds the newest policy rank 0 sent over the in-memory relay (engine_relay.py) so the
    server can serve it, and forwards agent uploads to rank 0, which folds them into its
    shard of the next epoch (training_zmq.rs:948-1058 -> REINFORCE.py:70-95)."""

    def __init__(self, spec: EngineSpec, obs_dim: int, act_dim: int, publish_dir: str,
                 save_model_path: Optional[str] = None):
        from ..ops.mlp import MLPSpec
        from .engine_relay import ApiRelay

        self.spec = spec
        self.publish_dir = publish_dir  # spec / result / logs of the child ranks (no weights)
        os.makedirs(publish_dir, exist_ok=True)
        self.save_model_path = save_model_path or os.path.join(os.getcwd(), "server_model.pt")
        self.obs_dim, self.act_dim = int(obs_dim), int(act_dim)
        self.hidden = int(spec.trainer.get("hidden", 128))
        self.discrete = spec.env != "HalfCheetahSynth-v0"
        g = torch.Generator().manual_seed(int(spec.trainer.get("seed", 0)))
        self.pi = MLPSpec(self.obs_dim, self.hidden, self.act_dim, not self.discrete).init(g)
        with_vf = bool(spec.trainer.get("with_baseline", True)) or spec.algo in ("a2c", "ppo")
        self.vf = MLPSpec(self.obs_dim, self.hidden, 1).init(g) if with_vf else None
        self.version = 0
        self.epoch = 0
        self.accepts_uploads = (bool(spec.trainer.get("agent_rows", True)) and spec.kind in ("vec", "host"))
        self.ignored_trajectories = 0
        self.relay = ApiRelay()
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)

    def set_model(self, blob) -> bool:
        """A model rank 0 sent (relay thread); True if it is newer than the one held."""
        with self._cv:
            if blob.version <= self.version:
                return False
            self.pi = torch.from_numpy(blob.pi)
            self.vf = None if blob.vf is None else torch.from_numpy(blob.vf)
            self.version = int(blob.version)
            self.epoch = int(blob.meta.get("epoch", blob.version))
            self._cv.notify_all()
        return True

    def wait_version(self, version: int, timeout: float) -> bool:
        with self._cv:
            return self._cv.wait_for(lambda: self.version >= version, timeout)

    def get_weights(self) -> Dict[str, Any]:
        with self._lock:
            w = {"pi": self.pi.clone(), "version": self.version, "obs_dim": self.obs_dim, "act_dim": self.act_dim,
                 "hidden": self.hidden, "discrete": self.discrete}
            if self.vf is not None:
                w["vf"] = self.vf.clone()
        return w

    def policy_module(self):
        from ..models.policies import build_policy_module

        w = self.get_weights()
        return build_policy_module(self.obs_dim, self.act_dim, self.hidden, w["pi"], w.get("vf"), self.discrete)

    def model_bytes(self) -> bytes:
        from ..models.policies import torchscript_bytes

        return torchscript_bytes(self.policy_module())

    def save(self, path: Optional[str] = None) -> None:
        from ..models.policies import export_torchscript

        export_torchscript(self.policy_module(), path or self.save_model_path)

    def receive_trajectory(self, trajectory) -> bool:
        """Forward an agent upload to rank 0 (queued until the ranks are up); the engine's own
        epochs publish the models, so this never reports an update."""
        if not self.accepts_uploads or not self.relay.send_upload(trajectory):
            self.ignored_trajectories += 1
        return False

    def train_model(self) -> None:
        raise RuntimeError("the ranks train in the child process; use TrainingServer.train()")

    def log_epoch(self) -> None:
        pass

    def close(self) -> None:
        self.relay.close()


class MultiRankEngineRunner:
    """Runs the engine's ranks as a ``torch.distributed.run`` child (one rank per GPU over
    RCCL); rank 0's models arrive over the relay and go straight to the server's store."""

    def __init__(self, algo: RemoteEngineAlgorithm, service, env_dir: str, t_start: float):
        self.algo = algo
        self.service = service
        self.env_dir = env_dir
        self.t_start = t_start
        self.result: Optional[TrainResult] = None
        self.error: Optional[BaseException] = None
        self._thread: Optional[threading.Thread] = None
        algo.relay.on_model(self._on_model)

    def _on_model(self, blob):
        if self.algo.set_model(blob):
            self.service.updates += 1
            self.service.publish_model()

    def train(self, epochs: Optional[int] = None, target_return: Optional[float] = None, window: int = 100,
              max_seconds: Optional[float] = None, log_every: int = 1, publish_every: int = 1) -> TrainResult:
        from .launcher import spawn_ranks

        spec_path = os.path.join(self.algo.publish_dir, "spec.json")
        with open(spec_path, "w") as f:
            f.write(self.algo.spec.to_json())
        res_path = os.path.join(self.algo.publish_dir, "result.json")
        if os.path.exists(res_path):
            os.remove(res_path)
        argv = ["engine", "--spec", spec_path, "--env-dir", self.env_dir,
                "--log-every", str(log_every), "--publish-every", str(publish_every), "--window", str(window),
                "--t-start-wall", repr(time.time() - (time.perf_counter() - self.t_start)), "--result", res_path,
                "--version0", str(self.algo.version)] + self.algo.relay.argv()
        if epochs is not None:
            argv += ["--epochs", str(epochs)]
        if target_return is not None:
            argv += ["--target-return", str(target_return)]
        if max_seconds is not None:
            argv += ["--max-seconds", str(max_seconds)]
        self.algo.relay.reset_control()  # no stale STOP / upload port of a previous run
        rc = spawn_ranks(argv, self.algo.spec.world_size)
        if rc != 0:
            raise RuntimeError(f"engine ranks exited with code {rc}")
        d = json.load(open(res_path))
        final = int(d.pop("version", self.algo.version))
        self.algo.wait_version(final, 10.0)  # the last MODEL frame is in flight over the relay
        self.result = TrainResult(**d)
        return self.result

    # background training (TrainingServer.train(background=True))
    def start(self, **kw):
        self.error = None

        def run():
            try:
                self.train(**kw)
            except BaseException as e:  # noqa: BLE001 -- surfaced by join()
                self.error = e

        self._thread = threading.Thread(target=run, name="relayrl-engine-ranks", daemon=True)
        self._thread.start()

    def stop(self):
        """Ask the ranks to stop after their current epoch (STOP over the relay; the ranks
        agree on it with one all-reduce per epoch)."""
        if self._thread is not None and self._thread.is_alive():
            self.algo.relay.send_stop()

    def join(self, timeout: Optional[float] = None) -> Optional[TrainResult]:
        if self._thread is not None:
            self._thread.join(timeout)
        if self.error is not None:
            raise self.error
        return self.result


def run_engine_rank(spec: EngineSpec, env_dir: str, epochs: Optional[int], target_return: Optional[float],
                    window: int, max_seconds: Optional[float], log_every: int, publish_every: int,
                    t_start_wall: Optional[float], result_path: Optional[str], relay_up: Optional[int] = None,
                    relay_down: Optional[int] = None, version0: int = 0) -> int:
    """One rank of a multi-GPU engine (``python -m relayrl_prototype_amd engine ...``).  Rank 0
    ends the relay (engine_relay.py): agent uploads in, models out, STOP."""
    from ..parallel.comm import Comm, dist_env, init_distributed, local_device_index

    _, _, world = dist_env()
    comm = init_distributed() if world > 1 else Comm()
    dev = None
    if torch.cuda.is_available():
        dev = torch.device("cuda", local_device_index())
        torch.cuda.set_device(dev)
    algo = EngineAlgorithm(spec, env_dir, comm=comm, device=dev)
    algo.version = int(version0)
    relay = None

    class _Pub:
        """Rank 0 sends every new policy to the API process from memory.  The snapshot is an
        asynchronous copy into pinned memory (EngineAlgorithm.weights_async) and goes out at
        the NEXT publish, once the copy is done: no stream drain per published epoch; flush()
        sends the last one."""
        updates = 0
        pending = None

        def publish_model(self):
            if relay is not None and algo.publishes_policy:
                prev, self.pending = self.pending, algo.weights_async()
                if prev is not None:
                    self._send(prev.result())

        def flush(self):
            if self.pending is not None:
                self._send(self.pending.result())
                self.pending = None

        @staticmethod
        def _send(w):
            from .model_store import ModelBlob

            meta = {k: w[k] for k in ("obs_dim", "act_dim", "hidden", "discrete")}
            meta["epoch"] = w.get("epoch", algo.epoch)
            relay.send_model(ModelBlob(int(w["version"]), meta, w["pi"].numpy(),
                                       None if w.get("vf") is None else w["vf"].numpy()))

    # the clock of the threshold metric starts where the API object was built (parent process)
    t_start = time.perf_counter() - (time.time() - t_start_wall) if t_start_wall else time.perf_counter()
    pub = _Pub()
    r = EngineRunner(algo, pub, t_start)
    if relay_up is not None and comm.rank == 0:
        from .engine_relay import RankRelay

        relay = RankRelay(relay_up, relay_down, algo.receive_trajectory, r.stop)
    r.agree_stop = relay_up is not None and comm.multi  # STOP reaches rank 0 only
    res = r.train(epochs, target_return, window, max_seconds, log_every, publish_every)
    pub.flush()  # the last snapshot (the final version the API process waits for)
    if algo.rank == 0 and result_path:
        tmp = result_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(dict(res.to_dict(), version=algo.version), f)
        os.replace(tmp, result_path)
    if relay is not None:
        relay.close()
    if hasattr(algo.trainer, "close"):
        algo.trainer.close()
    elif hasattr(algo.trainer, "finish"):
        algo.trainer.finish()
    if comm.enabled:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0
