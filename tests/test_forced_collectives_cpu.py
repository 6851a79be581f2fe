"""``RRL_FORCE_COLLECTIVES=1`` on the CPU (gloo): a one-rank group takes the world > 1 code
path (``Comm.multi``) -- reduce -> all_reduce -> Adam -- and trains to the same weights as
the plain world-1 path (fp32 summation order aside).  gloo cannot be captured, so
``graph_safe`` is False there; the GPU twin (tests/test_forced_collectives_gpu.py) checks the
captured RCCL form."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SNIPPET = r"""
import json, torch
from relayrl_prototype_amd.parallel.comm import Comm, init_distributed
from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer
comm = init_distributed()
out = {"multi": comm.multi, "world": comm.world, "backend": comm.backend, "graph_safe": comm.graph_safe}
res = []
for c in (comm, Comm(collectives=False)):
    cfg = HostTrainerConfig(num_envs=16, rollout_len=8, with_baseline=True, train_vf_iters=3, num_threads=1,
                            gamma=0.98, lam=0.97, seed=4)
    tr = HostVecTrainer(cfg, c, device="cpu")
    for _ in range(3):
        tr.train_epoch()
    tr.finish()
    res.append((tr.learner.pi.params.clone(), tr.learner.vf.params.clone(), c.multi))
out["multi_paths"] = [r[2] for r in res]
out["pi_maxdiff"] = float((res[0][0] - res[1][0]).abs().max())
out["vf_maxdiff"] = float((res[0][1] - res[1][1]).abs().max())
import torch.distributed as dist
dist.destroy_process_group()
print(json.dumps(out))
"""


def test_forced_one_rank_group_takes_the_multi_rank_path():
    env = dict(os.environ, RRL_FORCE_COLLECTIVES="1", RRL_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-c", SNIPPET], env=env, capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["multi"] and out["world"] == 1 and out["backend"] == "gloo" and not out["graph_safe"], out
    assert out["multi_paths"] == [True, False], out
    assert out["pi_maxdiff"] < 1e-5 and out["vf_maxdiff"] < 1e-5, out
