"""hipGraph captures under the two hazards that can break them in a long-running server
(VERDICT r4 item 7):

* Python's garbage collector running finalizers INSIDE a capture (an automatic collection
  triggered by an allocation in the captured code): every capture runs with automatic
  collection paused (utils/tracing.gc_paused).  Here the collector is made to run as often
  as possible (threshold 1) over cycles whose finalizers record and synchronise CUDA events.
* Another thread issuing HIP calls (synchronous copies) while a capture is open: captures
  use ``capture_error_mode="thread_local"`` (PG learner epoch, value loop, Pong update), so
  the other thread's calls neither fail nor invalidate the capture.

Every captured run must replay and be BITWISE equal to the eager run of the same seeds."""
import contextlib
import gc
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


class _Cycle:
    """Garbage only the cycle collector frees; its finalizer synchronises on the device."""

    def __init__(self, dev):
        self.me = self
        self.st = torch.cuda.Stream(dev)
        self.ev = torch.cuda.Event()
        self.t = torch.zeros(16, device=dev)

    def __del__(self):
        self.ev.record(self.st)
        self.ev.synchronize()


@contextlib.contextmanager
def _gc_pressure(dev):
    old = gc.get_threshold()
    gc.set_threshold(1, 1, 1)
    for _ in range(64):
        _Cycle(dev)
    try:
        yield
    finally:
        gc.set_threshold(*old)
        gc.collect()


def _run_vec(dev, graphs, epochs=4, **kw):
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    cfg = VecTrainerConfig(num_envs=1024, rollout_len=16, train_vf_iters=8, use_graphs=graphs, seed=3, **kw)
    tr = VecTrainer(cfg, device=dev)
    for _ in range(epochs):
        _Cycle(dev)  # fresh cyclic garbage before every epoch (and its captures)
        _Cycle(dev)
        tr.train_epoch()
    torch.cuda.synchronize()
    vg = len(tr.learner.vloop._graphs)
    return tr.pi.params.clone(), tr.vf.params.clone(), tr.learner.graph_replays, vg


def _run_pong(dev, graphs, epochs=4):
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    tr = PixelA2CTrainer(PixelA2CConfig(num_envs=256, rollout_len=5, seed=2, use_graphs=graphs), device=dev)
    for _ in range(epochs):
        _Cycle(dev)
        tr.train_epoch()
    torch.cuda.synchronize()
    return tr.model.params.clone(), len(tr._graphs)


def test_pg_epoch_capture_survives_gc_finalizers(cuda):
    with _gc_pressure(cuda):
        e = _run_vec(cuda, False)
        g = _run_vec(cuda, True)
    assert g[2] >= 3 and e[2] == 0  # the whole-epoch graph replayed
    assert torch.equal(e[0], g[0]) and torch.equal(e[1], g[1])


def test_value_loop_capture_survives_gc_finalizers(cuda):
    # PPO with target_kl: the epoch is not capturable (host KL read), the value loop alone is
    kw = dict(algo="ppo", train_pi_iters=3, target_kl=10.0)
    with _gc_pressure(cuda):
        e = _run_vec(cuda, False, **kw)
        g = _run_vec(cuda, True, **kw)
    assert g[2] == 0 and g[3] >= 1 and e[3] == 0  # value-loop graphs, no whole-epoch graph
    assert torch.equal(e[0], g[0]) and torch.equal(e[1], g[1])


def test_pong_update_capture_survives_gc_finalizers(cuda):
    with _gc_pressure(cuda):
        e = _run_pong(cuda, False)
        g = _run_pong(cuda, True)
    assert g[1] >= 1 and e[1] == 0
    assert torch.equal(e[0], g[0])


@pytest.mark.parametrize("which", ["pong", "pg"])
def test_capture_with_another_thread_issuing_hip_copies(cuda, which):
    """A 'transport' thread does synchronous host<->device copies on its own stream for the
    whole run, including while the Pong update / PG epoch is being captured."""
    stop = threading.Event()
    errors, copies = [], [0]

    def transport():
        try:
            torch.cuda.set_device(cuda)
            s = torch.cuda.Stream(cuda)
            x = torch.randn(1 << 16)
            while not stop.is_set():
                with torch.cuda.stream(s):
                    y = x.to(cuda)
                    z = y.cpu()
                assert z.shape == x.shape
                copies[0] += 1
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    e = _run_pong(cuda, False) if which == "pong" else _run_vec(cuda, False)
    th = threading.Thread(target=transport, daemon=True)
    th.start()
    try:
        g = _run_pong(cuda, True) if which == "pong" else _run_vec(cuda, True)
    finally:
        stop.set()
        th.join(30)
    assert not errors, errors
    assert copies[0] > 0
    assert torch.equal(e[0], g[0])
    if which == "pong":
        assert g[1] >= 1
    else:
        assert g[2] >= 3 and torch.equal(e[1], g[1])
