"""Logger format, checkpoint round trip, reference-weight import, TB events, algorithms on CPU."""
import json
import os

import numpy as np
import pytest
import torch

from relayrl_prototype_amd.utils.checkpoint import import_reference_weights, load_checkpoint, save_checkpoint
from relayrl_prototype_amd.utils.logger import EpochLogger, read_progress, setup_logger_kwargs
from relayrl_prototype_amd.utils.tensorboard import EventWriter, ProgressTensorboard, crc32c, read_events

REF_CKPT = "/root/reference/examples/REINFORCE_without_baseline/classic_control/cartpole/zmq/client_model.pt"


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283


def test_epoch_logger_progress_format(tmp_path):
    kw = setup_logger_kwargs("relayrl-reinforce-info", seed=3, data_dir=str(tmp_path))
    assert kw["output_dir"].endswith(os.path.join("relayrl-reinforce-info", "relayrl-reinforce-info_s3"))
    lg = EpochLogger(**kw, quiet=True)
    lg.save_config({"a": 1, "b": [1, 2]})
    for ep in range(3):
        lg.store(EpRet=[1.0 + ep, 3.0 + ep], EpLen=5)
        lg.log_tabular("Epoch", ep + 1)
        lg.log_tabular("EpRet", with_min_and_max=True)
        lg.log_tabular("EpLen", average_only=True)
        lg.dump_tabular()
    cols = read_progress(os.path.join(kw["output_dir"], "progress.txt"))
    assert list(cols) == ["Epoch", "AverageEpRet", "StdEpRet", "MaxEpRet", "MinEpRet", "EpLen"]
    assert cols["AverageEpRet"] == [2.0, 3.0, 4.0] and cols["StdEpRet"][0] == 1.0
    assert json.load(open(os.path.join(kw["output_dir"], "config.json")))["exp_name"] == "relayrl-reinforce-info"


def test_reference_progress_parses():
    p = ("/root/reference/examples/REINFORCE_without_baseline/box2d/lunar_lander/grpc/logs/relayrl-reinforce-info/"
         "relayrl-reinforce-info_s298690001/progress.txt")
    if not os.path.exists(p):
        pytest.skip("reference not mounted")
    cols = read_progress(p)
    assert len(cols["Epoch"]) == 118 and "DeltaLossPi" in cols


def test_checkpoint_roundtrip(tmp_path):
    st = {"pi": {"params": torch.randn(10), "step": torch.tensor([3], dtype=torch.int32)}, "epoch": 7,
          "cfg": {"lr": 0.1, "name": "x"}}
    save_checkpoint(str(tmp_path / "c"), st)
    back = load_checkpoint(str(tmp_path / "c"))
    assert torch.equal(back["pi"]["params"], st["pi"]["params"]) and back["epoch"] == 7
    assert back["cfg"]["name"] == "x"


def test_import_reference_weights_without_unpickling():
    if not os.path.exists(REF_CKPT):
        pytest.skip("reference not mounted")
    pi, vf = import_reference_weights(REF_CKPT, 4, 2, 128)
    assert pi.size == 17410 and vf is None and np.isfinite(pi).all()
    from relayrl_prototype_amd.models.cpu_policy import CPUPolicy

    p = CPUPolicy(4, 2, 128, True, pi)
    act, data = p.step(np.zeros(4, np.float32), np.ones(2, np.float32))
    assert act.shape == (1,) and np.isfinite(data["logp_a"]).all()


def test_event_writer_and_progress_tail(tmp_path):
    w = EventWriter(str(tmp_path / "tb"))
    w.add_scalar("loss", 1.5, 3)
    w.close()
    assert read_events(w.path) == [("loss", 1.5, 3)]
    logs = tmp_path / "logs" / "exp" / "exp_s0"
    logs.mkdir(parents=True)
    (logs / "progress.txt").write_text("Epoch\tAverageEpRet\tLossPi\n1\t10.0\t0.5\n2\t20.0\t0.25\n")
    tb = ProgressTensorboard(str(tmp_path / "logs"), ["AverageEpRet", "LossPi"])
    assert tb.poll_once() == 4
    ev = glob_events(logs / "tb")
    assert ("AverageEpRet", 20.0, 2) in read_events(ev)


def glob_events(d):
    import glob

    return glob.glob(os.path.join(str(d), "events.out.tfevents.*"))[0]


@pytest.mark.parametrize("algo,discrete", [("REINFORCE", True), ("PPO", True), ("PPO", False), ("A2C", True)])
def test_trajectory_algorithms_cpu(tmp_path, monkeypatch, algo, discrete):
    """Each algorithm ingests synthetic episodes and produces finite updates (oracle path)."""
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    from relayrl_prototype_amd.algorithms.registry import make_algorithm
    from relayrl_prototype_amd.types import RelayRLAction, RelayRLTrajectory

    D, A = 3, 2
    alg = make_algorithm(algo, env_dir=str(tmp_path), config_path=str(tmp_path / "c.json"), obs_dim=D, act_dim=A,
                         buf_size=10000, device="cpu", traj_per_epoch=2, train_vf_iters=2, discrete=discrete,
                         train_pi_iters=3, hidden=64)
    p0 = alg.learner.pi.params.clone()
    rng = np.random.default_rng(0)
    updated = False
    for ep in range(2):
        t = RelayRLTrajectory(100, None)
        for s in range(7):
            act = np.array([rng.integers(0, A)]) if discrete else rng.standard_normal(A).astype(np.float32)
            t.add_action(RelayRLAction(obs=rng.standard_normal(D), act=act, mask=np.ones(A), rew=1.0,
                                       data={"logp_a": np.float32(-0.7 if discrete else -2.0)}, done=(s == 6)))
        updated = alg.receive_trajectory(t)
    assert updated and alg.epoch == 1
    assert torch.isfinite(alg.learner.pi.params).all() and not torch.equal(p0, alg.learner.pi.params)
    m = alg.last_metrics
    assert np.isfinite(m["LossPi"]) and np.isfinite(m["LossV"])
    alg.save(str(tmp_path / "m.pt"))
    assert os.path.getsize(tmp_path / "m.pt") > 1000


def test_phase_timer_and_roctx():
    from relayrl_prototype_amd.utils.tracing import PhaseTimer, roctx_available, roctx_range

    t = PhaseTimer(None)
    with t.phase("A"):
        with roctx_range("inner"):
            sum(range(1000))
    cols = t.columns()
    assert "AWallMs" in cols and cols["AWallMs"] >= 0
    assert isinstance(roctx_available(), bool)


def test_fault_injection_drop_and_corrupt(tmp_path, monkeypatch):
    """Corrupted uploads are rejected by the server, dropped ones show up as sequence gaps."""
    import time

    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.runtime.learner_service import LearnerService
    from relayrl_prototype_amd.transport.zmq_transport import ZmqTrainingEndpoint
    from relayrl_prototype_amd.types import RelayRLAction, RelayRLTrajectory
    from relayrl_prototype_amd.utils import faults

    class Alg:
        def __init__(self):
            self.got = []

        def get_weights(self):
            return {"pi": torch.zeros(3), "vf": None, "version": 0, "obs_dim": 1, "act_dim": 1, "hidden": 1,
                    "discrete": True}

        def model_bytes(self):
            return b""

        def receive_trajectory(self, t):
            self.got.append(t.seq)
            return False

    svc = LearnerService(Alg())
    svc.start()
    ep = ZmqTrainingEndpoint(svc, "tcp://127.0.0.1:0", "tcp://127.0.0.1:0")
    push = _native.ZmtpSocket(_native.SockType.PUSH)
    push.connect(f"tcp://127.0.0.1:{ep.traj_port}")
    inj = faults.reset("corrupt=1.0,seed=1")
    t = RelayRLTrajectory(10, None, agent_id="a")
    t.add_action(RelayRLAction(obs=np.zeros(2), rew=1.0, done=True))
    push.send([inj.filter_upload(t.encode())], 2000)
    inj = faults.reset("drop=1.0")
    t.seq = 1
    assert inj.filter_upload(t.encode()) is None
    faults.reset("")
    t.seq = 2
    push.send([t.encode()], 2000)
    t0 = time.time()
    while svc.received < 1 and time.time() - t0 < 10:
        time.sleep(0.01)
    assert ep.bad_frames == 1
    assert svc.algorithm.got == [2]
    t.seq = 5
    push.send([t.encode()], 2000)
    t0 = time.time()
    while svc.received < 2 and time.time() - t0 < 10:
        time.sleep(0.01)
    assert svc.dropped_seq == 2  # seq 3 and 4 never arrived
    push.close()
    ep.close()
    svc.stop()


def test_plot_utils(tmp_path):
    from relayrl_prototype_amd.utils.plot import get_datasets, get_newest_dataset, make_plots

    for s in range(2):
        d = tmp_path / "exp" / f"exp_s{s}"
        d.mkdir(parents=True)
        (d / "progress.txt").write_text("Epoch\tAverageEpRet\n" + "".join(f"{i}\t{i * (s + 1)}.0\n" for i in range(5)))
    runs = get_datasets(str(tmp_path))
    assert len(runs) == 2 and runs[0]["AverageEpRet"].iloc[4] == 4.0
    assert list(runs[1]["Unit"].unique()) == [1] and (runs[0]["Performance"] == runs[0]["AverageEpRet"]).all()
    assert get_newest_dataset(str(tmp_path), return_file_root=True).endswith("exp_s1")
    assert list(get_newest_dataset(str(tmp_path)).columns) == ["Epoch", "AverageEpRet"]
    out = tmp_path / "curve.png"
    make_plots([str(tmp_path) + "/"], xaxis="Epoch", values=["AverageEpRet"], smooth=2, out=str(out))
    assert out.exists() and out.stat().st_size > 1000


def test_plot_selects_runs_by_name_from_a_logs_tree(tmp_path):
    """prefixes, --select / --exclude, --legend, --count and --est as in the
    reference CLI (plot.py:178-253)."""
    import json as _json

    from relayrl_prototype_amd.utils.plot import get_all_datasets, main, plot_data

    logs = tmp_path / "logs"
    for name, scale in (("relayrl-reinforce-info", 1), ("relayrl-reinforce-vf-info", 2), ("relayrl-ppo-info", 3)):
        for seed in range(2):
            d = logs / name / f"{name}_s{seed}"
            d.mkdir(parents=True)
            (d / "config.json").write_text(_json.dumps({"exp_name": name}))
            (d / "progress.txt").write_text("Epoch\tEnvSteps\tAverageEpRet\n" + "".join(
                f"{i}\t{1000 * i}\t{scale * i + seed}.0\n" for i in range(6)))
    data = get_all_datasets([str(logs / "relayrl-reinforce")], verbose=False)  # a prefix: both reinforce dirs
    assert sorted({d["Condition1"].iloc[0] for d in data}) == ["relayrl-reinforce-info", "relayrl-reinforce-vf-info"]
    data = get_all_datasets([str(logs / "relayrl-")], select=["vf"], verbose=False)
    assert {d["Condition1"].iloc[0] for d in data} == {"relayrl-reinforce-vf-info"} and len(data) == 2
    data = get_all_datasets([str(logs / "relayrl-")], exclude=["vf", "ppo"], legend=["base"], verbose=False)
    assert {d["Condition1"].iloc[0] for d in data} == {"base"}
    assert sorted(d["Condition2"].iloc[0] for d in data) == ["base-0", "base-1"]
    with pytest.raises(ValueError):
        get_all_datasets([str(logs / "relayrl-")], legend=["a"], verbose=False)
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig = plt.figure()
    conds = plot_data(get_all_datasets([str(logs / "relayrl-")], select=["reinforce"], verbose=False),
                      xaxis="EnvSteps", value="Performance", condition="Condition2", estimator=np.max, ax=fig.gca())
    assert len(conds) == 4  # --count: one curve per run
    out = tmp_path / "two.png"
    main([str(logs / "relayrl-reinforce"), "--legend", "no-vf", "vf", "-y", "AverageEpRet", "--est", "max",
          "--smooth", "1", "--out", str(out)])
    assert out.exists() and out.stat().st_size > 1000


def test_server_config_manager(tmp_path, monkeypatch):
    monkeypatch.setenv("RRL_QUIET_CONFIG", "1")
    from relayrl_prototype_amd.utils.addresses import ServerConfigManager

    m = ServerConfigManager(str(tmp_path / "cfg.json"), {"training_server": {"host": "*", "port": 7000}})
    ts = m.get("training_server")
    assert ts.bind_address().endswith("0.0.0.0:7000") and ts.connect_address().endswith("127.0.0.1:7000")
    m.assign_free_ports()
    ports = {e["port"] for e in m.as_dict().values()}
    assert len(ports) == 3 and all(int(p) > 0 for p in ports)


def test_solved_check_window_of_100_episodes():
    """bench.py's time-to-threshold criterion: mean of the newest >= 100 finished episodes
    (whole epochs), NaN until 100 have finished; older epochs are dropped."""
    import math

    from relayrl_prototype_amd.runtime.vec_trainer import SolvedCheck

    c = SolvedCheck(475.0, min_episodes=100)
    assert math.isnan(c.update(30, 30 * 480.0))
    assert math.isnan(c.update(40, 40 * 470.0))
    m = c.update(50, 50 * 490.0)  # 120 episodes: all three epochs
    assert abs(m - (30 * 480 + 40 * 470 + 50 * 490) / 120) < 1e-9 and c.solved(m)
    m = c.update(120, 120 * 400.0)  # the newest epoch alone fills the window
    assert m == 400.0 and not c.solved(m) and len(c.hist) == 1
    assert math.isnan(SolvedCheck().update(0, 0.0))


def test_learner_service_evicts_silent_agents_and_endpoint_stops_pushing():
    import time as _t

    from relayrl_prototype_amd.runtime.learner_service import LearnerService

    class _Algo:
        def get_weights(self):
            import torch

            return {"pi": torch.zeros(4), "version": 0, "obs_dim": 1, "act_dim": 1, "hidden": 1, "discrete": True}

        def model_bytes(self):
            return b""

        def receive_trajectory(self, t):
            return False

    svc = LearnerService(_Algo())
    hooked = []
    svc.on_evict(hooked.extend)
    svc.register_agent("A")
    svc.register_agent("B")
    svc.agents["A"]["last_seen"] -= 100.0  # silent for 100 s
    assert svc.evict_stale(30.0) == ["A"] and hooked == ["A"]
    assert "A" in svc.evicted and list(svc.agents) == ["B"]
    svc.register_agent("A")  # a returning agent re-registers
    assert "A" in svc.agents
    svc.agents["B"]["last_seen"] -= 100.0
    svc.start_sweeper(30.0, period_s=0.05)
    t0 = _t.time()
    while "B" in svc.agents and _t.time() - t0 < 5:
        _t.sleep(0.02)
    svc.stop_sweeper()
    assert "B" not in svc.agents and "B" in hooked
