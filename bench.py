#!/usr/bin/env python3
"""Flagship benchmark: CartPole-v1 REINFORCE (+ value baseline), env steps/sec (whole node)
+ wall-clock to the return threshold.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  For N > 1 the driver
launches it under ``torch.distributed.run`` (one rank per GPU, RCCL); run WITHOUT a launcher
and ``--gpus N > 1``, this script starts ``torch.distributed.run`` itself as a CHILD process
(nothing touches the GPU first; never an exec) and relays rank 0's JSON line.

One "step" is one full training epoch of the on-device actor + learner
(runtime/vec_trainer.py): a rollout of num_envs x rollout_len env steps per GPU (policy
forward + sampling + env physics in one fused kernel) + value forward + GAE scan + 1 policy
Adam step + 80 value Adam steps (the reference REINFORCE.train_model, REINFORCE.py:97-125),
with one RCCL all-reduce of the flat gradient per optimiser step across ranks.  Nothing is
skipped inside the timed region.  Weak scaling: per-GPU envs are fixed as N grows.

BASELINE.md: the reference publishes no numbers, so ``vs_baseline`` is null.  The second
half of the metric, wall-clock to CartPole-v1 solved (mean return of the newest >= 100
episodes >= 475), is measured through the reference API -- the clock starts at
``TrainingServer(..., engine="vec")`` construction and stops at the first epoch that meets
the criterion -- with the tuned config AND the reference hyperparameters (gamma .98, lam .97,
pi lr 3e-4, V lr 1e-3, 80 value iterations), median over seeds, after the timed steps.
``benchmarks/reference_equivalent_cpu.py`` (the reference's per-step CPU pipeline, same
criterion) runs concurrently in a child process and is reported next to them.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

METRIC = "env steps/sec (whole node) + wall-clock to return threshold, CartPole REINFORCE"
REPO = os.path.dirname(os.path.abspath(__file__))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--num-envs", type=int, default=32768, help="envs per GPU")
    ap.add_argument("--rollout-len", type=int, default=64)
    ap.add_argument("--no-baseline", action="store_true", help="REINFORCE without the value baseline")
    ap.add_argument("--vf-iters", type=int, default=80)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu = plumbing check of the multi-rank path with the host engine (not a benchmark)")
    ap.add_argument("--ttt", action="store_true",
                    help="also measure wall-clock to the threshold with several ranks (default: one GPU only)")
    ap.add_argument("--no-ttt", action="store_true", help="skip the time-to-threshold measurement")
    ap.add_argument("--multi-ttt-seeds", type=int, default=2,
                    help="world > 1: seeds of each time-to-threshold measurement (the whole-node record carries "
                         "both halves of the metric; one GPU uses --ttt-seeds / --ttt-ref-seeds)")
    ap.add_argument("--preflight-deadline-s", type=float, default=90.0,
                    help="world > 1: deadline of the collective preflight (parallel/preflight.py: RCCL init, "
                         "70 KB all-reduce, P2P ring, a captured all-reduce replayed 3x vs eager); a node that "
                         "fails the capture part runs with eager collectives, one that fails RCCL reports it")
    # tuned TTT defaults: tools/ttt_sweep.py --grid r2 / r2refine (round 2, 10 seeds): 256 envs x 64 steps,
    # 10 value iterations, pi lr 2e-2 (median 9.8 ms after construction vs 13.7 ms for the round-1 1024 x 64,
    # 5 iterations, pi lr 1e-2)
    ap.add_argument("--ttt-envs", type=int, default=256)
    ap.add_argument("--ttt-rollout-len", type=int, default=64)
    ap.add_argument("--ttt-vf-iters", type=int, default=10)
    ap.add_argument("--ttt-ref-envs", type=int, default=512,
                    help="batch shape of the reference-hyperparameter TTT runs (tools/ttt_sweep.py --grid refhp: "
                         "512 x 16 was the fastest of 256..4096 envs x 16..128 steps)")
    ap.add_argument("--ttt-ref-rollout-len", type=int, default=16)
    ap.add_argument("--ttt-pi-lr", type=float, default=2e-2)
    ap.add_argument("--ttt-vf-lr", type=float, default=1e-2)
    ap.add_argument("--ttt-graphs", action="store_true",
                    help="capture the value loop as a hipGraph in the tuned TTT runs (eager is faster there: "
                         "the capture costs ~0.45 ms in the first epoch, tools/ttt_graph_probe.py)")
    ap.add_argument("--ttt-seeds", type=int, default=10, help="report the median over this many seeds")
    ap.add_argument("--ttt-ref-seeds", type=int, default=5, help="seeds of the reference-hyperparameter TTT")
    ap.add_argument("--ttt-max-s", type=float, default=30.0, help="give up on a seed after this many seconds")
    ap.add_argument("--ref-cpu-seconds", type=float, default=150.0,
                    help="budget of the concurrent reference-equivalent CPU run (0 = skip)")
    ap.add_argument("--phase-steps", type=int, default=3,
                    help="extra epochs AFTER the timed steps with HIP-event phase timing on (per-rank "
                         "Rollout / ValueFwd / Scan / Optimize / AllReduce ms); 0 = skip")
    ap.add_argument("--actor-learner", choices=("auto", "on", "off"), default="auto",
                    help="secondary phase: the actor -> learner-group P2P data plane (BASELINE config #3 "
                         "topology, K = 2 actor blocks per learner shard); auto = only with world > 1")
    ap.add_argument("--host-steps", type=int, default=6,
                    help="1 GPU: also time the host-env data path (C++ env threads + the C++ rollout driver, "
                         "cartpole-reinforce-host preset, lag-1 overlap) for this many epochs; 0 = skip")
    ap.add_argument("--pong-steps", type=int, default=20,
                    help="1 GPU: also time the A2C Pong pixel update (BASELINE config #4: Nature CNN on bf16 MFMA, "
                         "2048 envs x 5 steps) for this many updates; 0 = skip")
    ap.add_argument("--pong-big-envs", type=int, default=8192,
                    help="1 GPU: also time the A2C Pong update at this many envs (the six rollout forwards are "
                         "latency-bound at 2048 frames per launch); 0 = skip")
    ap.add_argument("--convergence", choices=("auto", "on", "off"), default="auto",
                    help="1 GPU: wall-clock / env steps to the return thresholds of BASELINE configs #3-#5 "
                         "(benchmarks/convergence_bench.py: A2C PongSynth, REINFORCE-with-baseline LunarLanderSynth, "
                         "PPO HalfCheetahSynth); auto = on with one GPU")
    ap.add_argument("--conv-seeds", type=int, default=3, help="seeds of each convergence preset (median reported)")
    ap.add_argument("--conv-budget-s", type=float, default=30.0, help="wall-clock budget per convergence run")
    ap.add_argument("--al-steps", type=int, default=10)
    ap.add_argument("--al-warmup", type=int, default=5)
    ap.add_argument("--al-env", default="LunarLanderSynth-v0")
    ap.add_argument("--al-num-envs", type=int, default=2048)
    ap.add_argument("--al-rollout-len", type=int, default=128)
    ap.add_argument("--al-vf-iters", type=int, default=80)
    ap.add_argument("--al-deadline-s", type=float, default=150.0,
                    help="wall-clock bound of the secondary actor-learner phase (then: recorded as failed)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------- launcher (no GPU here)
def spawn_ranks(argv) -> int:
    """torch.distributed.run as a CHILD (one rank per GPU, 127.0.0.1 rendezvous); its stdout is
    inherited, so rank 0's JSON line is this process's output."""
    import socket

    a = parse(argv)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = REPO + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------- time to threshold
def _ttt_config_file(tmp: str) -> str:
    import socket

    from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT

    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    for k in ("training_server", "trajectory_server", "agent_listener"):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        cfg["server"][k]["port"] = str(s.getsockname()[1])
        s.close()
    p = os.path.join(tmp, "relayrl_config.json")
    with open(p, "w") as f:
        json.dump(cfg, f)
    return p


def time_to_threshold(hp: dict, mi355x: dict, seeds: int, max_s: float, comm, threshold: float = 475.0):
    """Per seed: the clock starts at TrainingServer(..., engine="vec") construction (BASELINE.md:
    "from TrainingServer start") and stops after the first epoch whose newest >= 100 finished
    episodes average >= threshold (gymnasium CartPole-v1).  Returns (median s, per-seed s,
    median epochs, median env steps)."""
    import statistics

    import torch

    from relayrl_prototype_amd.api.server import TrainingServer

    os.environ.setdefault("RRL_QUIET_CONFIG", "1")
    times, epochs, steps = [], [], []
    with tempfile.TemporaryDirectory() as tmp:
        cfgp = _ttt_config_file(tmp)
        for seed in range(1, seeds + 1):
            h = dict(hp, seed=seed)
            h.update({k: v for k, v in mi355x.items()})
            comm.barrier()
            torch.cuda.synchronize()
            srv = TrainingServer("REINFORCE", 4, 2, 1000, env_dir=os.path.join(tmp, f"env{seed}"), config_path=cfgp,
                                 server_type="local", hyperparams=h, engine="vec")
            try:
                r = srv.train(target_return=threshold, window=100, max_seconds=max_s, log_every=0, publish_every=0)
            finally:
                srv.close(save=False)
            times.append(r.time_to_threshold_s if r.solved else float("inf"))
            epochs.append(r.epochs)
            steps.append(r.env_steps)
    med = statistics.median(times)
    return (None if med == float("inf") else med), times, int(statistics.median(epochs)), int(statistics.median(steps))


def start_reference_cpu(seconds: float):
    if seconds <= 0:
        return None
    cmd = [sys.executable, os.path.join(REPO, "benchmarks", "reference_equivalent_cpu.py"), "--seconds",
           str(seconds), "--window", "100"]
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env["HIP_VISIBLE_DEVICES"] = ""  # CPU only: never touches the GPU
    env["CUDA_VISIBLE_DEVICES"] = ""
    return subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)


def collect_reference_cpu(proc, budget_s: float):
    if proc is None:
        return None
    try:
        out, _ = proc.communicate(timeout=budget_s + 60)
    except subprocess.TimeoutExpired:
        proc.kill()
        return None
    for line in reversed(out.strip().splitlines()):
        try:
            return json.loads(line)
        except ValueError:
            continue
    return None


# ---------------------------------------------------------------------- host-env data path
def host_path_probe(steps: int, comm) -> dict:
    """The north-star data path on one GPU: CartPole envs stepped by C++ threads on the host,
    the T-step loop in C++ (csrc/runtime/host_rollout.cpp: zero-copy sampling launches), the
    same fused learner on the GPU, rollout k+1 overlapped with update k (lag 1).  Reported
    next to the headline; 2 untimed warmup epochs, then ``steps`` timed ones."""
    import torch

    from relayrl_prototype_amd.runtime.launcher import PRESETS, _make_trainer

    p = PRESETS["cartpole-reinforce-host"]
    dev = torch.device("cuda", torch.cuda.current_device())
    rec = {"preset": p.name, "steps": steps, "warmup": 2}
    tr = None
    try:
        tr = _make_trainer(p, comm, dev, {})
        for _ in range(2):
            tr.train_epoch()
        tr.finish()
        m0 = tr.metrics()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.train_epoch()
        tr.finish()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m1 = tr.metrics()
        n = m1["EnvSteps"] - m0["EnvSteps"]
        rec.update(env_steps_per_s=round(n / dt, 1), ms_per_epoch=round(dt / steps * 1e3, 3),
                   num_envs=tr.cfg.num_envs, rollout_len=tr.cfg.rollout_len, env_threads=tr.cfg.num_threads,
                   overlap=tr.overlap, per_env_step_us={k: round(v, 2) for k, v in m1.items()
                                                        if k.startswith("Host") and k.endswith("Us")})
    except Exception as e:  # noqa: BLE001 -- recorded; the headline still prints
        rec["error"] = f"{type(e).__name__}: {e}"[:300]
    finally:
        if tr is not None:
            tr.close()
            del tr
        torch.cuda.empty_cache()
    return rec


def pong_probe(steps: int, num_envs: int = 2048) -> dict:
    """BASELINE config #4 on one GPU: A2C on PongSynth-v0 pixels (Nature CNN, bf16 MFMA: the
    fused conv-stack forward and conv backward kernels of csrc/kernels/cnn_fused.hip, the fc
    GEMMs of csrc/kernels/fc.hip), ``num_envs`` envs x 5 steps per update, the whole update
    captured as one hipGraph; 3 untimed warmup updates, then ``steps`` timed ones.  Reported
    next to the headline."""
    import torch

    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    rec = {"config": f"A2C PongSynth-v0, Nature-CNN, {num_envs} envs x 5 steps", "steps": steps, "warmup": 3,
           "dtype": "bf16 (fp32 accumulate, fp32 master weights)"}
    tr = None
    try:
        cfg = PixelA2CConfig(num_envs=num_envs, rollout_len=5)
        tr = PixelA2CTrainer(cfg, device=torch.device("cuda", torch.cuda.current_device()))
        for _ in range(3):
            tr.train_epoch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.train_epoch()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rec.update(env_steps_per_s=round(steps * cfg.num_envs * cfg.rollout_len / dt, 1),
                   ms_per_update=round(dt / steps * 1e3, 3))
    except Exception as e:  # noqa: BLE001 -- recorded; the headline still prints
        rec["error"] = f"{type(e).__name__}: {e}"[:300]
    finally:
        del tr
        torch.cuda.empty_cache()
    return rec


def convergence_probe(seeds: int, budget_s: float) -> dict:
    """BASELINE configs #3-#5 learn: per preset and seed, the wall-clock (from trainer
    construction) and env steps at which the mean return of the newest >= 100 finished
    episodes first reaches each threshold (benchmarks/convergence_bench.py); the median over
    seeds per threshold (None if any seed missed it within the budget).  The full curves live
    in profiles/ (convergence_bench.py --out)."""
    import statistics

    import torch

    from benchmarks.convergence_bench import CONV, run

    out = {}
    for name in ("pong-a2c", "lunarlander-reinforce-baseline", "halfcheetah-ppo"):
        runs = []
        for seed in range(1, seeds + 1):
            try:
                r = run(name, {}, 0, budget_s, 10 ** 9, seed)
            except Exception as e:  # noqa: BLE001 -- recorded; the headline still prints
                runs.append({"error": f"{type(e).__name__}: {e}"[:300]})
                continue
            finally:
                torch.cuda.empty_cache()
            runs.append(r)
        ok = [r for r in runs if "error" not in r]
        rec = {"note": CONV[name]["note"], "seeds": seeds, "budget_s": budget_s,
               "overrides": ok[0]["overrides"] if ok else None}
        th = {}
        for t in CONV[name]["thresholds"]:
            hits = [r["thresholds"].get(str(t)) for r in ok]
            done = len(hits) == seeds and all(h is not None for h in hits)
            th[str(t)] = {"median_s": round(statistics.median(h["s"] for h in hits), 3) if done else None,
                          "median_env_steps": int(statistics.median(h["env_steps"] for h in hits)) if done else None,
                          "per_seed_s": [None if h is None else h["s"] for h in hits]}
        rec["thresholds"] = th
        rec["last_window_ret"] = [r["last_window_ret"] for r in ok]
        errs = [r["error"] for r in runs if "error" in r]
        if errs:
            rec["errors"] = errs
        out[name] = rec
    return out


# ---------------------------------------------------------------------- comm-phase observability
def phase_probe(tr, comm, steps: int) -> dict:
    """``steps`` more epochs with the trainer's HIP-event PhaseTimer on (after the timed
    region, so the headline number carries no event overhead).  Returns per-rank lists of
    per-epoch device ms per phase (AllReduce = every RCCL gradient / statistics all-reduce)."""
    tm = tr.timer
    tm.reset()
    tm.enabled = True
    if comm.world > 1:
        comm.timer = tm
    for _ in range(steps):
        tr.train_epoch()
    mine = tm.per_step(steps)
    tm.enabled = False
    comm.timer = None
    tm.reset()
    rows = comm.all_gather_object(mine)
    keys = sorted({k for r in rows for k in r})
    return {k: [r.get(k) for r in rows] for k in keys}


def actor_learner_probe(args, comm, on_gpu: bool) -> dict:
    """Secondary phase at world > 1: the actor -> learner data plane of BASELINE config #3.

    Every rank acts; ranks 0 .. W/2-1 also learn (learner_ranks = W/2, so K = 2 actor
    blocks per learner shard): each learner receives one remote rollout over P2P straight
    into its contiguous shard batch (C1, reference trajectory.rs:69-90 ->
    training_zmq.rs:948-1058), the shards all-reduce gradients inside the learner group,
    and each learner P2P-sends the new weights back to its remote actor (C2,
    training_zmq.rs:876-934 -> agent_zmq.rs:625-698) with a one-version lag (max_lag 1).
    Every received rollout header is verified (version within the lag, weight checksum of
    that version).  Errors and timeouts land in the record instead of failing the headline."""
    import torch

    from relayrl_prototype_amd.runtime.actor_learner import ActorLearner, ActorLearnerConfig

    W = comm.world
    L = max(1, W // 2)
    rec = {"env": args.al_env, "K": (W // L), "L": L, "world": W, "max_lag": 1, "steps": args.al_steps,
           "warmup": args.al_warmup}
    try:
        if on_gpu:
            n, t, vi, thr = args.al_num_envs, args.al_rollout_len, args.al_vf_iters, 8
        else:  # gloo plumbing check: tiny shapes, oracle ops
            n, t, vi, thr = 16, 8, 2, 1
        cfg = ActorLearnerConfig(env=args.al_env, num_envs=n, rollout_len=t, with_baseline=True, gamma=0.98,
                                 lam=0.97, pi_lr=3e-4, vf_lr=1e-3, train_vf_iters=vi, learner_ranks=L,
                                 learner_acts=True, max_lag=1, verify_versions=True, stall_timeout_s=0.0,
                                 num_threads=thr, seed=1)
        dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
        al = ActorLearner(cfg, comm, dev)
        rec.update(num_envs=n, rollout_len=t, train_vf_iters=vi, role="learner" if al.is_learner else "actor")
        sync = torch.cuda.synchronize if on_gpu else (lambda: None)
        for _ in range(args.al_warmup):
            al.step()
        comm.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.al_steps):
            al.step()
        comm.barrier()
        sync()
        dt_local = time.perf_counter() - t0
        dt = torch.tensor([dt_local], dtype=torch.float64, device=dev)
        comm.all_reduce_max_(dt)
        dt = float(dt.item())
        # phase timing in extra steps (events + the per-step syncs of verify_versions)
        al.timer.enabled = True
        ph_steps = max(2, args.al_steps // 2)
        for _ in range(ph_steps):
            al.step()
        phases = al.timer.per_step(ph_steps)
        al.timer.enabled = False
        al.finish()
        vers = al.last_hdr[:, 7].tolist() if al.is_learner and al.last_hdr is not None else []
        ok = all(al.version - 1 - cfg.max_lag <= v <= al.version - 1 for v in vers)
        per_rank = comm.all_gather_object({"rank": comm.rank, "role": rec["role"], "step_ms":
                                           round(dt_local / args.al_steps * 1e3, 3), "versions": vers,
                                           "versions_ok": ok, **phases})
        rec.update(
            env_steps_per_s=round(args.al_steps * t * n * len(al.topo.actors) / dt, 1),
            ms_per_step=round(dt / args.al_steps * 1e3, 3),
            versions_ok=all(r["versions_ok"] for r in per_rank),
            gather_ms=[r.get("GatherMs") for r in per_rank],
            allreduce_ms=[r.get("AllReduceMs") for r in per_rank],
            allreduce_calls=[r.get("AllReduceCalls") for r in per_rank],
            weight_send_ms=[r.get("WeightSendMs") for r in per_rank],
            weight_recv_ms=[r.get("WeightRecvMs") for r in per_rank],
            learn_ms=[r.get("LearnMs") for r in per_rank],
            rollout_ms=[r.get("RolloutMs") for r in per_rank],
            per_rank=per_rank,
            backend=comm.backend)
        al.watchdog.close()
    except Exception as e:  # noqa: BLE001 -- recorded, the headline line still prints
        rec["error"] = f"{type(e).__name__}: {e}"[:500]
    return rec


DEADLINE_EXIT = 3  # a hung secondary phase: the record still prints, the run reads as failed


def _arm_deadline(seconds: float, rank: int, emit, cleanup=None):
    """Timer thread: after ``seconds`` rank 0 runs ``emit`` (prints the JSON line with the
    phase marked failed) and every rank leaves with status DEADLINE_EXIT (non-zero, so
    torchrun and CI see the hang) -- a rank blocked inside a collective cannot be unwound,
    and each rank's own timer fires, so torchrun sees the whole group exit.  ``cleanup``
    (e.g. terminating the reference-CPU child) runs first."""
    import threading

    def fire():
        try:
            if cleanup is not None:
                cleanup()
            if rank == 0:
                emit()
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(DEADLINE_EXIT)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


# ---------------------------------------------------------------------- main
def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        return spawn_ranks(argv)
    if world_env is not None and int(world_env) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world_env} but --gpus {args.gpus}; launch one rank per GPU")
    import torch

    from relayrl_prototype_amd.parallel.comm import init_distributed, local_device_index

    on_gpu = args.device == "gpu"
    preflight = None
    if int(world_env or 1) > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if os.environ.get("RRL_PREFLIGHT", "1") != "0":
            # before this process touches the GPU: prove RCCL + graph capture in child processes
            from relayrl_prototype_amd.parallel.comm import local_device_index
            from relayrl_prototype_amd.parallel.preflight import run_preflight

            pf_backend = os.environ.get("RRL_DIST_BACKEND") or ("nccl" if on_gpu else "gloo")
            preflight = run_preflight(pf_backend, local_device_index(), args.preflight_deadline_s)
            if preflight is not None and not preflight["rccl_ok"]:
                if int(os.environ.get("RANK", "0")) == 0:
                    bad = [r for r in preflight["per_rank"] if not r.get("rccl_ok")]
                    print(json.dumps({"metric": METRIC, "value": None, "unit": "env_steps/s", "n_gpus": int(world_env),
                                      "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
                                      "scaling": "weak", "vs_baseline": None,
                                      "error": "collective preflight failed: " + "; ".join(
                                          f"rank {r['rank']} at {r.get('stage')}: {r.get('error')}" for r in bad[:4]),
                                      "preflight": preflight}), flush=True)
                return 2
            if preflight is not None and not preflight["graphs_ok"]:
                args.no_graphs = True  # eager collectives everywhere (value loop, TTT runs)
                args.ttt_graphs = False
        # a hung peer becomes an exception inside 90 s (recorded in the JSON by the secondary
        # actor-learner phase) instead of a 10-minute wait or a torn-down process
        os.environ.setdefault("RRL_COLLECTIVE_TIMEOUT_S", "90")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
    comm = init_distributed()
    world = comm.world
    rank = comm.rank
    ref_proc = start_reference_cpu(args.ref_cpu_seconds) if (rank == 0 and world == 1 and on_gpu) else None
    if on_gpu:
        torch.cuda.set_device(local_device_index())
        from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

        cfg = VecTrainerConfig(num_envs=args.num_envs, rollout_len=args.rollout_len,
                               with_baseline=not args.no_baseline, train_vf_iters=args.vf_iters,
                               use_graphs=not args.no_graphs)
        tr = VecTrainer(cfg, comm)
        sync = torch.cuda.synchronize
        dev = "cuda"
    else:
        from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

        cfg = HostTrainerConfig(num_envs=args.num_envs, rollout_len=args.rollout_len,
                                with_baseline=not args.no_baseline, train_vf_iters=args.vf_iters, num_threads=1,
                                gamma=0.98, lam=0.97)
        tr = HostVecTrainer(cfg, comm, device="cpu")
        sync = lambda: None  # noqa: E731
        dev = "cpu"
    for _ in range(args.warmup):
        tr.train_epoch()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_epoch()
    comm.barrier()
    sync()
    dt_local = time.perf_counter() - t0
    t = torch.tensor([dt_local], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(t)
    dt = float(t.item())
    m = tr.metrics()
    steps_per_epoch = cfg.num_envs * cfg.rollout_len * world
    value = steps_per_epoch * args.steps / dt
    per_rank = comm.all_gather_object(round(cfg.num_envs * cfg.rollout_len * args.steps / dt_local, 1))
    per_rank_ms = comm.all_gather_object(round(dt_local / args.steps * 1e3, 3))
    phases = phase_probe(tr, comm, args.phase_steps) if args.phase_steps > 0 else None
    host_rec = host_path_probe(args.host_steps, comm) if (on_gpu and world == 1 and args.host_steps > 0) else None
    pong_rec = pong_probe(args.pong_steps) if (on_gpu and world == 1 and args.pong_steps > 0) else None
    pong_big = (pong_probe(args.pong_steps, args.pong_big_envs)
                if (on_gpu and world == 1 and args.pong_steps > 0 and args.pong_big_envs > 0) else None)
    conv = None
    if on_gpu and (args.convergence == "on" or (args.convergence == "auto" and world == 1)):
        conv = convergence_probe(args.conv_seeds, args.conv_budget_s)

    def record(al_rec, ttt=None, ttt_ref=None, ref_cpu=None, do_ttt=False):
        """The ONE JSON line (rank 0)."""
        algo = "REINFORCE" if args.no_baseline else "REINFORCE-with-baseline"
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env_steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",  # value / policy steps: 3-way bf16 split of every fp32 operand (bf16x6), fp32-accurate
            "data": ("synthetic (on-device CartPole-v1 physics, random-init weights)" if on_gpu else
                     "CPU plumbing check of the multi-rank path (host engine, oracle ops) -- not a benchmark"),
            "config": {
                "model": f"{algo} MLP[128,128] CartPole-v1 (rollout: fp32 MFMA; policy and value steps: "
                         "fp32-accurate bf16x6 split MFMA, csrc/kernels/value_grad.hip)",
                "global_batch": steps_per_epoch,
                "seq_len": cfg.rollout_len,
                "parallelism": f"dp{world}",
                "envs_per_gpu": cfg.num_envs,
                "train_vf_iters": cfg.train_vf_iters if cfg.with_baseline else 0,
                "hyperparams": "reference defaults (gamma .98, lam .97, pi_lr 3e-4, vf_lr 1e-3)",
            },
            "backend": comm.backend,
            "rccl_world": world if comm.backend == "nccl" else 0,
            # collectives / optimiser loops replayed from hipGraphs (False: eager, e.g. after a failed
            # capture preflight or over gloo)
            "graphs": bool(cfg.use_graphs and comm.graph_safe) if on_gpu else False,
            "per_rank_env_steps_per_s": per_rank,
            "per_rank_ms_per_step": per_rank_ms,
            "final_avg_ep_ret": None if m["AverageEpRet"] != m["AverageEpRet"] else round(m["AverageEpRet"], 2),
        }
        if do_ttt:
            def pack(r, hp, shape_cfg, seeds):
                return {"time_to_threshold_s": None if r[0] is None else round(r[0], 4),
                        "per_seed_s": [round(x, 4) if x != float("inf") else None for x in r[1]],
                        "epochs": r[2], "env_steps": r[3], "seeds": seeds, "hyperparams": hp, **shape_cfg}

            shape_cfg = {"num_envs": args.ttt_envs, "rollout_len": args.ttt_rollout_len}
            rec["time_to_threshold_s"] = None if ttt[0] is None else round(ttt[0], 4)
            rec["time_to_threshold_reference_hparams_s"] = None if ttt_ref[0] is None else round(ttt_ref[0], 4)
            rec["time_to_threshold"] = {
                "criterion": "mean return of the newest >= 100 finished episodes >= 475 (gymnasium CartPole-v1), "
                             "checked after every epoch (its sums read one epoch behind, behind the next queued "
                             "epoch: RRL_TTT_LAGGED_CHECK; the clock stops when they reach the host)",
                "clock": "starts at TrainingServer(..., engine='vec') construction (api/server.py), stops after "
                         "the first solved epoch; includes trainer/buffer allocation",
                "tuned": pack(ttt, {"gamma": 0.99, "lam": 0.95, "pi_lr": args.ttt_pi_lr, "vf_lr": args.ttt_vf_lr,
                                    "train_vf_iters": args.ttt_vf_iters}, shape_cfg, args.ttt_seeds),
                "reference_hparams": pack(ttt_ref, {"gamma": 0.98, "lam": 0.97, "pi_lr": 3e-4, "vf_lr": 1e-3,
                                                    "train_vf_iters": 80},
                                          {"num_envs": args.ttt_ref_envs, "rollout_len": args.ttt_ref_rollout_len},
                                          args.ttt_ref_seeds),
            }
        if phases is not None:
            rec["phase_ms_per_step"] = dict(phases, steps=args.phase_steps,
                                            note="per rank, device ms per epoch from HIP events, measured in "
                                                 "extra epochs after the timed region")
        if host_rec is not None:
            rec["host_env_path"] = host_rec
        if pong_rec is not None:
            rec["pong_a2c"] = pong_rec
        if pong_big is not None:
            rec["pong_a2c_big"] = pong_big
        if conv is not None:
            rec["convergence"] = dict(conv, criterion="mean return of the newest >= 100 finished episodes >= "
                                      "threshold, checked every epoch; clock from trainer construction",
                                      data="synthetic device envs (docs/ENVS.md), random-init weights")
        if al_rec is not None:
            rec["actor_learner"] = al_rec
        if preflight is not None:
            rec["preflight"] = preflight
        if ref_cpu is not None:
            rec["reference_equivalent_cpu"] = {
                "env_steps_per_s": round(ref_cpu.get("value", 0.0), 1),
                "time_to_threshold_s": ref_cpu.get("time_to_threshold_s"),
                "best_window_return": ref_cpu.get("best_window_return"),
                "budget_s": args.ref_cpu_seconds,
                "criterion": "same (newest >= 100 episodes >= 475), reference hyperparameters, batch-1 per-step "
                             "TorchScript pipeline on one CPU thread, measured concurrently in this run",
                "source": "benchmarks/reference_equivalent_cpu.py"}
        return rec

    al_rec = None
    if args.actor_learner == "on" or (args.actor_learner == "auto" and world > 1):
        # a hung RCCL transfer in the secondary phase must not cost the headline: past the
        # deadline rank 0 prints the line with the phase marked failed and every rank exits
        guard = _arm_deadline(args.al_deadline_s, rank, lambda: print(json.dumps(record(
            {"error": f"deadline: actor-learner phase did not finish within {args.al_deadline_s} s",
             "exit_status": DEADLINE_EXIT})), flush=True),
            cleanup=(lambda: ref_proc.kill()) if ref_proc is not None else None)
        try:
            al_rec = actor_learner_probe(args, comm, on_gpu)
        finally:
            guard.cancel()
    ttt = ttt_ref = None
    do_ttt = on_gpu and not args.no_ttt
    if do_ttt and world > 1:  # the whole-node record carries both halves of the metric
        args.ttt_seeds = args.ttt_ref_seeds = args.multi_ttt_seeds
    if do_ttt:
        del tr
        torch.cuda.empty_cache()
        tuned = {"with_vf_baseline": True, "train_vf_iters": args.ttt_vf_iters, "pi_lr": args.ttt_pi_lr,
                 "vf_lr": args.ttt_vf_lr, "gamma": 0.99, "lam": 0.95}
        ref_hp = {"with_vf_baseline": True, "train_vf_iters": 80, "pi_lr": 3e-4, "vf_lr": 1e-3, "gamma": 0.98,
                  "lam": 0.97}
        shape = {"num_envs": args.ttt_envs, "rollout_len": args.ttt_rollout_len}
        ttt = time_to_threshold(tuned, dict(shape, use_graphs=bool(args.ttt_graphs)), args.ttt_seeds,
                                args.ttt_max_s, comm)
        ref_shape = {"num_envs": args.ttt_ref_envs, "rollout_len": args.ttt_ref_rollout_len}
        ttt_ref = time_to_threshold(ref_hp, dict(ref_shape, use_graphs=not args.no_graphs), args.ttt_ref_seeds,
                                    args.ttt_max_s, comm)
    ref_cpu = collect_reference_cpu(ref_proc, args.ref_cpu_seconds)
    if rank == 0:
        print(json.dumps(record(al_rec, ttt, ttt_ref, ref_cpu, do_ttt)), flush=True)
    if comm.enabled:
        import torch.distributed as dist

        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001 -- after a recorded comm failure
            pass
    return 0


if __name__ == "__main__":
    if os.environ.get("WORLD_SIZE"):
        # under torchrun: a rank's exception lands in the launcher's failure summary (the root
        # cause's traceback, not only "exitcode 1"), which is the tail a failed run shows
        from torch.distributed.elastic.multiprocessing.errors import record

        main = record(main)
    sys.exit(main())
