"""bench.py's multi-rank contract on CPU: ``python bench.py --gpus 2`` without an external
launcher starts torch.distributed.run as a child (gloo here, RCCL on MI355X) and prints ONE
JSON line for the whole job."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    return r


def test_bench_spawns_ranks_without_torchrun():
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu", "--num-envs", "16",
              "--rollout-len", "8", "--vf-iters", "2"], {"RRL_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["steps"] == 2 and rec["warmup"] == 1 and rec["backend"] == "gloo"
    assert rec["config"]["global_batch"] == 2 * 16 * 8
    assert len(rec["per_rank_env_steps_per_s"]) == 2
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    for k in ("metric", "unit", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert k in rec
    # comm-phase observability: per-rank phase lists, AllReduce included
    ph = rec["phase_ms_per_step"]
    assert len(ph["AllReduceMs"]) == 2 and all(x > 0 for x in ph["AllReduceMs"])
    assert ph["AllReduceCalls"] == [4.0, 4.0]  # stats + policy + 2 value steps
    # secondary phase: actor -> learner-group P2P fan-in / weight fan-out, lag 1, headers verified
    al = rec["actor_learner"]
    assert "error" not in al, al
    assert al["K"] == 2 and al["L"] == 1 and al["versions_ok"] is True
    assert al["env_steps_per_s"] > 0 and al["gather_ms"][0] > 0 and al["weight_recv_ms"][1] is not None
    vers = al["per_rank"][0]["versions"]
    assert len(vers) == 2 and vers[0] - vers[1] == 1  # own rollout on v_k, the remote actor's on v_{k-1}


def test_bench_rejects_world_size_mismatch():
    r = _run(["--gpus", "2", "--device", "cpu"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_actor_learner_deadline_keeps_the_headline():
    """A secondary phase that overruns its deadline (a hung transfer) still yields ONE JSON line
    with the headline and the phase marked failed, and the run exits NON-zero (bench.DEADLINE_EXIT
    on every rank) so torchrun / CI see the hang."""
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "1", "--device", "cpu", "--num-envs", "16",
              "--rollout-len", "8", "--vf-iters", "2", "--phase-steps", "0", "--al-steps", "100000",
              "--al-deadline-s", "3"], {"RRL_DIST_BACKEND": "gloo"})
    assert r.returncode != 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and rec["n_gpus"] == 2
    assert rec["actor_learner"]["error"].startswith("deadline")
    assert rec["actor_learner"]["exit_status"] == 3


def _line(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    return json.loads(lines[0])


_SMALL = ["--gpus", "2", "--steps", "1", "--warmup", "1", "--device", "cpu", "--num-envs", "16", "--rollout-len", "8",
          "--vf-iters", "2", "--phase-steps", "0", "--actor-learner", "off"]


def test_preflight_capture_failure_falls_back_to_eager_collectives():
    """the collective preflight runs in child processes before the ranks touch the
    device; a failed graph-capture check turns graphs off and the run still yields a valid line."""
    r = _run(_SMALL, {"RRL_DIST_BACKEND": "gloo", "RRL_PREFLIGHT_INJECT": "capture"})
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r)
    assert rec["value"] > 0 and rec["graphs"] is False
    pf = rec["preflight"]
    assert pf["rccl_ok"] is True and pf["graphs_ok"] is False and len(pf["per_rank"]) == 2
    assert all(p["stage"] in ("capture", "done") for p in pf["per_rank"])


def test_preflight_collective_failure_reports_instead_of_hanging():
    for inject, extra in (("rccl", []), ("hang", ["--preflight-deadline-s", "25"])):
        r = _run(_SMALL + extra, {"RRL_DIST_BACKEND": "gloo", "RRL_PREFLIGHT_INJECT": inject}, timeout=200)
        assert r.returncode != 0, (inject, r.stderr[-2000:])
        rec = _line(r)
        assert rec["value"] is None and rec["error"].startswith("collective preflight failed"), rec
        assert rec["preflight"]["rccl_ok"] is False
        if inject == "hang":
            stages = {p["stage"] for p in rec["preflight"]["per_rank"]}
            assert "timeout" in stages, rec["preflight"]
