"""Launcher / CLI: presets for the BASELINE configs, per-rank logging, checkpoint-resume,
and the multi-rank spawn (torch.distributed.run child, gloo on CPU)."""
import glob
import json
import os
import subprocess
import sys

import pytest

from relayrl_prototype_amd.runtime.launcher import PRESETS, run_preset

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_presets_cover_baseline_configs():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))["configs"]
    assert len(base) == 5 and len(PRESETS) >= 5
    # each BASELINE config -> the preset that runs it, checked on the config's own words
    cover = {0: ("cartpole-reinforce-zmq", ("CartPole", "ZMQ")),
             1: ("cartpole-reinforce-baseline", ("REINFORCE-with-baseline", "CartPole")),
             2: ("lunarlander-reinforce-baseline", ("LunarLander", "RCCL")),
             3: ("pong-a2c", ("A2C", "Pong")),
             4: ("halfcheetah-ppo", ("PPO", "HalfCheetah"))}
    for i, (name, words) in cover.items():
        assert name in PRESETS, name
        for w in words:
            assert w in base[i], (i, w)
    assert PRESETS["cartpole-reinforce-zmq"].overrides["server_type"] == "zmq"
    assert PRESETS["cartpole-reinforce-baseline"].overrides["with_baseline"] is True
    assert PRESETS["lunarlander-reinforce-baseline"].overrides["env"].startswith("LunarLander")
    assert PRESETS["halfcheetah-ppo"].overrides["algo"] == "ppo"
    assert PRESETS["pong-a2c"].kind == "pixel"
    kinds = {p.kind for p in PRESETS.values()}
    assert kinds == {"agent_server", "vec", "actor_learner", "pixel", "host"}


def test_pixel_preset_cpu_logs_and_resumes(tmp_path, monkeypatch):
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    ov = {"num_envs": 2, "rollout_len": 2, "seed": 3}
    m = run_preset("pong-a2c", 2, str(tmp_path), ov, checkpoint_every=2)
    assert m["Updates"] == 2 and m["EnvSteps"] == 8
    prog = glob.glob(str(tmp_path / "**" / "progress.txt"), recursive=True)
    assert prog and "EnvStepsPerSec" in open(prog[0]).readline()
    ck = str(tmp_path / "pong-a2c_ckpt_r0")
    assert os.path.exists(os.path.join(ck, "state.json"))
    m2 = run_preset("pong-a2c", 1, str(tmp_path / "r"), ov, resume=ck)
    assert m2["Updates"] == 3  # resumed counters


def test_cli_spawns_ranks_gloo(tmp_path):
    env = dict(os.environ, PYTHONPATH=REPO, RRL_QUIET_CONFIG="1", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "relayrl_prototype_amd", "train", "--preset", "pong-a2c", "--gpus", "2",
                        "--epochs", "1", "--out", str(tmp_path), "--set", "num_envs=2", "rollout_len=2"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    assert json.loads(line)["EnvSteps"] == 2 * 2 * 2  # whole job over 2 ranks


def test_rank_failure_group_restart_resumes(tmp_path):
    """Rank 1 crashes after epoch 2; torchrun restarts the group, every rank resumes from
    its own checkpoint and the run completes all epochs (SURVEY §5.3 elastic recovery)."""
    env = dict(os.environ, PYTHONPATH=REPO, RRL_QUIET_CONFIG="1", OMP_NUM_THREADS="1", RRL_FAULT_KILL="1:2")
    r = subprocess.run([sys.executable, "-m", "relayrl_prototype_amd", "train", "--preset", "pong-a2c", "--gpus", "2",
                        "--epochs", "4", "--out", str(tmp_path), "--checkpoint-every", "1", "--auto-resume",
                        "--max-restarts", "1", "--set", "num_envs=2", "rollout_len=2"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert os.path.exists(tmp_path / ".fault_fired_r1_e2")
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    m = json.loads(line)
    assert m["Updates"] == 4 and m["EnvSteps"] == 4 * 2 * 2 * 2


def test_stalled_actor_group_restart_resumes(tmp_path):
    """Actor-learner preset over 3 gloo ranks: rank 2 hangs before epoch 3; the other
    ranks' step watchdogs exit them (EXIT_STALL) well inside the collective timeout,
    torchrun restarts the group and every rank resumes from its checkpoint."""
    env = dict(os.environ, PYTHONPATH=REPO, RRL_QUIET_CONFIG="1", OMP_NUM_THREADS="1", RRL_FAULT_STALL="2:3:120")
    r = subprocess.run([sys.executable, "-m", "relayrl_prototype_amd", "train", "--preset",
                        "lunarlander-reinforce-baseline", "--gpus", "3", "--epochs", "4", "--out", str(tmp_path),
                        "--checkpoint-every", "1", "--auto-resume", "--max-restarts", "1", "--set", "num_envs=4",
                        "rollout_len=8", "train_vf_iters=2", "num_threads=1", "stall_timeout_s=4"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert os.path.exists(tmp_path / ".stall_fired_r2_e3")
    assert "[watchdog]" in r.stderr and "stalled" in r.stderr
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    assert json.loads(line)["EnvSteps"] == 4 * 8 * 4 * 3


def _worker_agree_resume(rank, world, port, ckroot, q):
    try:
        import torch

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        torch.set_num_threads(1)
        from relayrl_prototype_amd.parallel.comm import init_distributed
        from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer
        from relayrl_prototype_amd.runtime.launcher import _agree_resume, ckpt_dir
        from relayrl_prototype_amd.utils.checkpoint import save_checkpoint

        comm = init_distributed(backend="gloo")
        cfg = HostTrainerConfig(num_envs=8, rollout_len=8, hidden=32, train_vf_iters=1, num_threads=1, seed=rank)
        # rank 0 trained to epoch 3, rank 1's checkpoint is a stale epoch-1 state (it was evicted)
        tr = HostVecTrainer(cfg, comm, device="cpu")
        with torch.no_grad():
            tr.learner.pi.params.add_(float(rank + 1))
        save_checkpoint(ckpt_dir(ckroot, "p", rank), {"trainer": tr.state_dict(), "epoch": 3 if rank == 0 else 1})
        comm.barrier()
        fresh = HostVecTrainer(cfg, comm, device="cpu")
        start = _agree_resume(fresh, comm, ckpt_dir(ckroot, "p", rank))
        g = [torch.zeros_like(fresh.learner.pi.params) for _ in range(world)]
        torch.distributed.all_gather(g, fresh.learner.pi.params)
        q.put((rank, start, bool(torch.equal(g[0], g[1]))))
        torch.distributed.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e), False))


def test_auto_resume_ranks_agree_on_one_epoch(tmp_path):
    """ranks holding checkpoints of different epochs all resume at the newest one,
    with the learner state of the rank that holds it (no mismatched collectives)."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_agree_resume, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    assert res == [(0, 3, True), (1, 3, True)], res
