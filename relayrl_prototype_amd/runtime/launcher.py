"""Launcher: one process per GPU, named presets for the five BASELINE.json configurations.

    python -m relayrl_prototype_amd train --preset cartpole-reinforce-baseline --gpus 1 --epochs 50
    python -m relayrl_prototype_amd train --preset pong-a2c --gpus 8 --epochs 2000

``--gpus N > 1`` outside torchrun starts ``torch.distributed.run`` as a CHILD process
(never an exec, nothing touches the GPU before it) with a 127.0.0.1 rendezvous, and
returns its exit code; each rank then runs ``run_preset``.  The reference has no
launcher (one Python process per TrainingServer, training_server_wrapper.rs); its only
multi-process story was N agents over TCP (config 1 here).

Every preset logs the reference's progress.txt columns plus throughput columns through
``EpochLogger`` (rank 0) and can checkpoint / resume (utils/checkpoint.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Callable, Dict, Optional


@dataclass
class Preset:
    name: str
    baseline_config: str
    kind: str  # vec | host | actor_learner | pixel | agent_server
    overrides: Dict


PRESETS: Dict[str, Preset] = {
    "cartpole-reinforce-zmq": Preset(
        "cartpole-reinforce-zmq", "REINFORCE (no baseline) CartPole-v1, 1 agent <-> 1 trainer over ZMQ on CPU",
        "agent_server", {"env": "CartPole-v1", "server_type": "zmq", "episodes_per_epoch": 8}),
    "cartpole-reinforce-baseline": Preset(
        "cartpole-reinforce-baseline", "REINFORCE-with-baseline CartPole-v1, 1 actor+learner per MI355X",
        "vec", {"env": "CartPole-v1", "num_envs": 32768, "rollout_len": 64, "with_baseline": True}),
    "lunarlander-reinforce-baseline": Preset(
        "lunarlander-reinforce-baseline", "REINFORCE-with-baseline LunarLander, actor GPUs -> learner group "
        "(P2P rollout fan-in to learner shards, gradient all-reduce inside the group; default learner_ranks=0 = "
        "every rank learns its own rollout, K = 1 -- the fastest on one node; --set learner_ranks=L for L "
        "learner shards fed by W/L actor blocks each, as in bench.py's world > 1 actor-learner phase)",
        "actor_learner", {"env": "LunarLanderSynth-v0", "num_envs": 2048, "rollout_len": 128, "with_baseline": True,
                          "learner_acts": True, "learner_ranks": 0, "num_threads": 8}),
    "pong-a2c": Preset(
        "pong-a2c", "A2C Pong pixels, Nature-CNN on MFMA, DP gradient all-reduce",
        "pixel", {"num_envs": 1024, "rollout_len": 5}),
    "halfcheetah-ppo": Preset(
        "halfcheetah-ppo", "PPO HalfCheetah continuous Gaussian policy, large-batch GAE, HBM rollout buffer",
        "vec", {"env": "HalfCheetahSynth-v0", "algo": "ppo", "num_envs": 16384, "rollout_len": 256,
                "train_pi_iters": 10, "train_vf_iters": 10, "with_baseline": True, "gamma": 0.99, "lam": 0.95}),
    "halfcheetah-ppo-host": Preset(
        "halfcheetah-ppo-host", "PPO HalfCheetah with C++ host env threads (pinned H2D/D2H pipeline, "
        "lag-1 rollout/update overlap)",
        "host", {"env": "HalfCheetahSynth-v0", "algo": "ppo", "num_envs": 4096, "rollout_len": 256,
                 "train_pi_iters": 10, "train_vf_iters": 10, "num_threads": 16, "with_baseline": True,
                 "overlap": True}),
    "cartpole-reinforce-host": Preset(
        "cartpole-reinforce-host", "REINFORCE-with-baseline CartPole-v1 with C++ host env threads (pinned "
        "H2D/D2H pipeline, lag-1 rollout/update overlap)",
        "host", {"env": "CartPole-v1", "num_envs": 8192, "rollout_len": 64, "with_baseline": True,
                 "num_threads": 16, "gamma": 0.98, "lam": 0.97, "overlap": True}),
}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_trainer(preset: Preset, comm, device, overrides: Dict):
    kw = dict(preset.overrides)
    kw.update(overrides)
    if preset.kind == "vec":
        from .vec_trainer import VecTrainer, VecTrainerConfig

        return VecTrainer(VecTrainerConfig(**_filter(VecTrainerConfig, kw)), comm, device)
    if preset.kind == "host":
        from .host_trainer import HostTrainerConfig, HostVecTrainer

        return HostVecTrainer(HostTrainerConfig(**_filter(HostTrainerConfig, kw)), comm, device)
    if preset.kind == "actor_learner":
        from .actor_learner import ActorLearner, ActorLearnerConfig

        return ActorLearner(ActorLearnerConfig(**_filter(ActorLearnerConfig, kw)), comm, device)
    if preset.kind == "pixel":
        from .pixel_trainer import PixelA2CConfig, PixelA2CTrainer

        return PixelA2CTrainer(PixelA2CConfig(**_filter(PixelA2CConfig, kw)), comm, device)
    raise ValueError(preset.kind)


def _filter(cls, kw: Dict) -> Dict:
    import dataclasses

    names = {f.name for f in dataclasses.fields(cls)}
    return {k: v for k, v in kw.items() if k in names}


class EpochSnapshot:
    """The trainer's state at the START of the running epoch, kept on the device (elastic
    mode): learner parameters, Adam moments and step counters (+ device env state where the
    trainer has it) copied into preallocated buffers on the stream -- no host sync per epoch
    -- and the host counters.  A failure inside an epoch can leave k of its updates applied
    (a fault in the value loop's 40th all-reduce leaves 39 value steps and the policy step);
    the survivors restore this snapshot before they re-form, so the retried epoch starts
    from a consistent state, not from ``state_dict()`` of the broken
    trainer."""

    def __init__(self):
        self.bufs = None
        self.counters = None

    def take(self, tr) -> None:
        if not hasattr(tr, "snapshot_tensors"):
            return
        ts = tr.snapshot_tensors()
        if self.bufs is None or len(self.bufs) != len(ts) or any(
                b.shape != t.shape or b.device != t.device for b, t in zip(self.bufs, ts)):
            self.bufs = [t.detach().clone() for t in ts]
        else:
            for b, t in zip(self.bufs, ts):
                b.copy_(t.detach())
        self.counters = dict(tr.counters())

    @property
    def taken(self) -> bool:
        return self.counters is not None

    def restore(self, tr) -> None:
        import torch

        with torch.no_grad():
            for t, b in zip(tr.snapshot_tensors(), self.bufs):
                t.copy_(b)
        tr.set_counters(self.counters)


def _drop_graphs(tr) -> None:
    """Forget the captured graphs of a trainer whose process group broke: they hold RCCL
    collectives of the destroyed communicator."""
    for obj in (tr, getattr(tr, "learner", None)):
        if obj is not None and hasattr(obj, "drop_graphs"):
            obj.drop_graphs()


def _epoch(tr):
    if hasattr(tr, "train_epoch"):
        return tr.train_epoch()
    return tr.step()


def ckpt_dir(out_dir: str, name: str, rank: int) -> str:
    return os.path.join(out_dir, f"{name}_ckpt_r{rank}")


def _agree_resume(tr, comm, path: str) -> int:
    """Auto-resume that every rank agrees on: the job restarts from the NEWEST checkpoint
    epoch E any rank holds (all-reduce max).  Ranks whose own checkpoint is from epoch E load
    it (learner state + their env streams); the lowest such rank that can serve as a source
    (a learner for the actor-learner engine) then broadcasts the learner state, so ranks
    with a stale or missing checkpoint (e.g. one evicted by an elastic shrink before the
    restart) rejoin with fresh env streams but identical weights, and every rank runs the
    same epochs -- no mismatched collectives."""
    import torch

    from ..utils.checkpoint import load_checkpoint

    st = load_checkpoint(path) if os.path.exists(os.path.join(path, "state.json")) else None
    mine = int(st.get("epoch", 0)) if st is not None else -1
    if comm.world == 1:
        if st is not None:
            tr.load_state_dict(st["trainer"])
        return max(mine, 0)
    dev = torch.device("cuda", torch.cuda.current_device()) if comm.backend == "nccl" else torch.device("cpu")
    e = torch.tensor([float(mine)], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(e)
    E = int(e.item())
    if E < 0:
        return 0
    can_src = getattr(tr, "is_learner", True)
    cand = torch.tensor([float(comm.rank if (mine == E and can_src) else comm.world)], dtype=torch.float64,
                        device=dev)
    comm.all_reduce_min_(cand)
    src = int(cand.item())
    if src >= comm.world:
        raise RuntimeError(f"auto-resume: no learner rank holds the newest checkpoint (epoch {E})")
    if mine == E:
        tr.load_state_dict(st["trainer"])
    elif st is not None:
        print(f"[resume] rank {comm.rank}: own checkpoint is from epoch {mine}, the job resumes at {E}; "
              f"learner state from rank {src}", flush=True)
    if hasattr(tr, "sync_from_rank0"):
        tr.sync_from_rank0(src)
    return E


def run_preset(name: str, epochs: int, out_dir: str = "runs", overrides: Optional[Dict] = None,
               checkpoint_every: int = 0, resume: Optional[str] = None, log_every: int = 1,
               on_metrics: Optional[Callable[[Dict], None]] = None, auto_resume: bool = False,
               elastic: bool = False) -> Dict:
    """Run one rank of a preset until ``epochs`` epochs are done; returns the last metrics
    (rank 0).  Checkpoints are per rank (each rank owns its env streams); with
    ``auto_resume`` a (re)started rank continues from its own latest checkpoint, which is
    how a torchrun group restart after a rank failure recovers (--max-restarts).

    ``elastic``: a stalled rank does not stop the job -- the survivors' failed collective
    leads to a re-form of the process group without it (parallel/elastic.py), the trainer is
    rebuilt on the smaller group from its in-memory state (learner state broadcast from the
    new rank 0) and the failed epoch is retried.  An evicted rank returns
    ``{"Evicted": True}``."""
    import torch

    from ..parallel.comm import Comm, dist_env, init_distributed
    from ..utils.logger import EpochLogger, setup_logger_kwargs

    preset = PRESETS[name]
    overrides = dict(overrides or {})
    if preset.kind == "agent_server":
        return _run_agent_server(preset, epochs, out_dir, overrides)
    from ..parallel.comm import local_device_index

    orig_rank, _, world = dist_env()
    eg = None
    if elastic and world > 1:
        from ..parallel.elastic import ElasticGroup

        eg = ElasticGroup()
        comm = eg.init_group()
        # collective timeouts detect a stalled peer; the exiting step watchdog would end the
        # survivors too
        overrides.setdefault("stall_timeout_s", 0.0)
    else:
        comm = init_distributed() if world > 1 else Comm()
    if torch.cuda.is_available():
        dev = torch.device("cuda", local_device_index())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    tr = _make_trainer(preset, comm, dev, overrides)
    start = 0
    if auto_resume and resume is None:
        start = _agree_resume(tr, comm, ckpt_dir(out_dir, name, orig_rank))
    elif resume:
        from ..utils.checkpoint import load_checkpoint

        st = load_checkpoint(resume)
        tr.load_state_dict(st["trainer"])
    logger = None
    if comm.rank == 0:
        kw = setup_logger_kwargs(f"relayrl-{name}", seed=int(overrides.get("seed", 0)), data_dir=out_dir)
        logger = EpochLogger(**kw, quiet=True)
        logger.save_config({"preset": name, "overrides": overrides, "world_size": comm.world,
                            "baseline_config": preset.baseline_config})
    t0 = time.perf_counter()
    last: Dict = {}
    from ..utils.faults import maybe_kill_rank, maybe_stall_rank

    from ..utils.faults import set_context

    completed = False
    snap = EpochSnapshot() if eg is not None else None
    dump = os.environ.get("RRL_ELASTIC_DUMP") if eg is not None else None
    try:
        ep = start + 1
        while ep <= epochs:
            try:
                set_context(orig_rank if eg is not None else comm.rank, ep, out_dir)
                if snap is not None:
                    snap.take(tr)
                maybe_stall_rank(orig_rank if eg is not None else comm.rank, ep, out_dir)
                _epoch(tr)
                m = tr.metrics() if (ep % log_every == 0 or ep == epochs) else None
            except Exception as e:
                if eg is None:
                    raise
                from ..parallel.elastic import Evicted

                if hasattr(tr, "watchdog"):
                    tr.watchdog.close()
                if hasattr(tr, "finish") and not hasattr(tr, "watchdog"):
                    # a host trainer's rollout thread running ahead (its own envs, no peers)
                    try:
                        tr.finish()
                    except Exception:  # noqa: BLE001
                        pass
                if dump:
                    _dump_state(dump, f"failed_r{orig_rank}.pt", tr)
                # the epoch-start state, not the broken trainer's: the failed epoch may have
                # applied part of its updates before the collective that failed
                if snap is not None and snap.taken:
                    snap.restore(tr)
                sd = tr.state_dict()
                _drop_graphs(tr)
                # CU-masked streams / grid limit of the old trainer (host_trainer.close); no
                # finish(): that would wait on transfers of the broken group
                _release(tr, finish=False)
                try:
                    comm = eg.reform()
                except Evicted as ev:
                    print(f"[elastic] {ev}", flush=True)
                    eg.close()
                    return {"Evicted": True, "Epoch": ep - 1}
                if getattr(comm, "unchanged", False):
                    raise  # every rank is alive: not a lost peer
                if dump:
                    # the restored snapshot as a resumable checkpoint under the NEW rank: a
                    # fault-free run of the shrunken group resumed from it must end the retried
                    # epoch with the same weights (tests/test_elastic.py)
                    from ..utils.checkpoint import save_checkpoint

                    save_checkpoint(ckpt_dir(dump, name, comm.rank), {"trainer": sd, "epoch": ep - 1,
                                                                      "world": comm.world, "rank": comm.rank})
                print(f"[elastic] rank {orig_rank}: re-formed without the lost rank(s) after {type(e).__name__}; "
                      f"world {comm.world}, rank {comm.rank}, retrying epoch {ep}", flush=True)
                ov = dict(overrides)
                if preset.kind == "actor_learner":
                    from .actor_learner import Topology

                    req = dict(preset.overrides)
                    req.update(overrides)
                    if int(req.get("learner_ranks", 0)):
                        ov["learner_ranks"] = Topology.fit_learners(comm.world, int(req["learner_ranks"]),
                                                                    bool(req.get("learner_acts", True)))
                tr = _make_trainer(preset, comm, dev, ov)
                tr.load_state_dict(sd)
                if hasattr(tr, "sync_from_rank0"):
                    tr.sync_from_rank0()
                if comm.rank == 0 and logger is None:
                    kw = setup_logger_kwargs(f"relayrl-{name}", seed=int(overrides.get("seed", 0)), data_dir=out_dir)
                    logger = EpochLogger(**kw, quiet=True)
                continue
            if m is not None:
                el = time.perf_counter() - t0
                if comm.rank == 0 and m:
                    m = dict(m)
                    m["Time"] = el
                    if "EnvSteps" in m and el > 0:
                        m["EnvStepsPerSec"] = m["EnvSteps"] / el
                    m["UpdatesPerSec"] = (ep - start) / el if el > 0 else 0.0
                    if dev.type == "cuda":
                        m["HBMUsedGB"] = torch.cuda.max_memory_allocated(dev) / 2 ** 30
                    for k, v in m.items():
                        if isinstance(v, (int, float)):
                            logger.log_tabular(k, v)
                    logger.dump_tabular()
                    last = m
                    if on_metrics:
                        on_metrics(m)
            if checkpoint_every and ep % checkpoint_every == 0 and hasattr(tr, "state_dict"):
                from ..utils.checkpoint import save_checkpoint

                # keyed on the ORIGINAL (torchrun) rank: after an elastic shrink the survivors'
                # new ranks would overwrite other ranks' directories
                save_checkpoint(ckpt_dir(out_dir, name, orig_rank), {"trainer": tr.state_dict(), "epoch": ep,
                                                                     "world": comm.world, "rank": comm.rank})
            maybe_kill_rank(orig_rank, ep, out_dir)
            ep += 1
        completed = True
    finally:
        # also on an exception: a host trainer's CU limit is process-wide (host_trainer.close);
        # finish() (pending transfers) only after a clean run
        _release(tr, finish=completed)
    if eg is not None:
        last = dict(last)
        last["ElasticReforms"] = eg.reforms
        last["FinalWorld"] = comm.world
        eg.close()
    return last


def _dump_state(d: str, fname: str, tr) -> None:
    """Test hook (RRL_ELASTIC_DUMP): the broken trainer's learner state as it failed."""
    import torch

    os.makedirs(d, exist_ok=True)
    sd = tr.state_dict()
    torch.save(sd.get("learner", sd), os.path.join(d, fname))


def _release(tr, finish: bool = True) -> None:
    """close() (host trainer: CU-masked streams + the process-wide grid limit) or finish()."""
    if hasattr(tr, "close"):
        tr.close()
    elif finish and hasattr(tr, "finish"):
        tr.finish()


def _run_agent_server(preset: Preset, epochs: int, out_dir: str, overrides: Dict) -> Dict:
    """Config 1: TrainingServer + RelayRLAgent over ZMQ (or gRPC) in one process, CPU only."""
    import numpy as np

    from .. import _native
    from ..api.agent import RelayRLAgent
    from ..api.server import TrainingServer
    from ..config import DEFAULT_CONFIG_CONTENT

    os.makedirs(out_dir, exist_ok=True)
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(_free_port())
    per = int(overrides.get("episodes_per_epoch", preset.overrides["episodes_per_epoch"]))
    cfg["algorithms"]["REINFORCE"]["traj_per_epoch"] = per
    cfg_path = os.path.join(out_dir, "relayrl_config.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg, f, indent=2)
    st = overrides.get("server_type", preset.overrides["server_type"])
    srv = TrainingServer("REINFORCE", 4, 2, 1_000_000, env_dir=out_dir, config_path=cfg_path, server_type=st,
                         device="cpu")
    agent = RelayRLAgent(config_path=cfg_path, server_type=st)
    env = _native.VecEnv(overrides.get("env", "CartPole-v1"), 1, int(overrides.get("seed", 0)), 1)
    obs = np.zeros((1, env.obs_dim), np.float32)
    rew = np.zeros(1, np.float32)
    done = np.zeros(1, np.float32)
    act = np.zeros(1, np.int32)
    env.reset_ptr(obs.ctypes.data)
    steps, t0 = 0, time.perf_counter()
    try:
        for _ in range(epochs * per):
            r = 0.0
            while True:
                a = agent.request_for_action(obs[0], None, r)
                act[0] = int(np.asarray(a.get_act()).reshape(-1)[0])
                env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
                r = float(rew[0])
                steps += 1
                if done[0] > 0:
                    agent.flag_last_action(r)
                    break
        srv.wait_idle(60)
        el = time.perf_counter() - t0
        return {"EnvSteps": steps, "EnvStepsPerSec": steps / el, "Updates": srv.service.updates,
                "ModelVersion": agent.model_version}
    finally:
        agent.close()
        srv.close(save=True)


def spawn_ranks(argv, gpus: int, max_restarts: int = 0) -> int:
    """Start torch.distributed.run as a child with one rank per GPU; returns its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           f"--max-restarts={max_restarts}", "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "relayrl_prototype_amd"] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return subprocess.call(cmd, env=env)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="python -m relayrl_prototype_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("train", help="run a training preset (one process per GPU)")
    t.add_argument("--preset", choices=sorted(PRESETS), default="cartpole-reinforce-baseline")
    t.add_argument("--gpus", type=int, default=1)
    t.add_argument("--epochs", type=int, default=20)
    t.add_argument("--out", default="runs")
    t.add_argument("--set", nargs="*", default=[], help="overrides key=value (e.g. num_envs=8192)")
    t.add_argument("--checkpoint-every", type=int, default=0)
    t.add_argument("--resume", default=None)
    t.add_argument("--auto-resume", action="store_true", help="continue from this rank's last checkpoint if any")
    t.add_argument("--max-restarts", type=int, default=0, help="torchrun group restarts after a rank failure")
    t.add_argument("--elastic", action="store_true",
                   help="survivors of a stalled rank re-form the group without it and continue")
    e = sub.add_parser("engine", help="one rank of a TrainingServer device engine (runtime/engine.py)")
    e.add_argument("--spec", required=True)
    e.add_argument("--env-dir", default=".")
    e.add_argument("--relay-up", type=int, default=None, help="rank 0: port of the upload / control PULL")
    e.add_argument("--relay-down", type=int, default=None, help="rank 0: port of the API process's model PULL")
    e.add_argument("--version0", type=int, default=0, help="model version the API process holds")
    e.add_argument("--epochs", type=int, default=None)
    e.add_argument("--target-return", type=float, default=None)
    e.add_argument("--window", type=int, default=100)
    e.add_argument("--max-seconds", type=float, default=None)
    e.add_argument("--log-every", type=int, default=1)
    e.add_argument("--publish-every", type=int, default=1)
    e.add_argument("--t-start-wall", type=float, default=None)
    e.add_argument("--result", default=None)
    sub.add_parser("presets", help="list the presets")
    b = sub.add_parser("build", help="compile the HIP and C++ extensions in-tree")
    b.add_argument("--force", action="store_true")
    p = sub.add_parser("plot", help="plot progress.txt runs")
    p.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.cmd == "presets":
        for k, v in PRESETS.items():
            print(f"{k:34s} [{v.kind}] {v.baseline_config}")
        return 0
    if a.cmd == "build":
        from .._build import build

        build(force=a.force)
        return 0
    if a.cmd == "engine":
        from .engine import EngineSpec, run_engine_rank

        spec = EngineSpec.from_json(open(a.spec).read())
        return run_engine_rank(spec, a.env_dir, a.epochs, a.target_return, a.window, a.max_seconds, a.log_every,
                               a.publish_every, a.t_start_wall, a.result, a.relay_up, a.relay_down, a.version0)
    if a.cmd == "plot":
        from ..utils.plot import main as plot_main

        plot_main(a.rest)
        return 0
    in_torchrun = "LOCAL_RANK" in os.environ and "WORLD_SIZE" in os.environ
    if a.gpus > 1 and not in_torchrun:
        return spawn_ranks(argv, a.gpus, a.max_restarts)
    ov = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        try:
            v = json.loads(v)
        except ValueError:
            pass
        ov[k] = v
    m = run_preset(a.preset, a.epochs, a.out, ov, a.checkpoint_every, a.resume, auto_resume=a.auto_resume,
                   elastic=a.elastic)
    if m:
        print(json.dumps({k: v for k, v in m.items() if isinstance(v, (int, float, str))}), flush=True)
    return 0
