"""Frame-ring observations for PongSynth A2C (csrc/kernels/pong_render.h, pong.hip, cnn_fused.hip).

Each env step renders ONE new frame into a ring of frames and an observation is the 4 store rows
of its frames; the conv kernels interleave the 4 frames into the s2d channel order as they load
them.  Every test here compares against the 4-frame observation path bitwise: the ring changes
where the bytes come from, not one value the network sees.
"""
import pytest
import torch

from relayrl_prototype_amd.models.nature_cnn import FC_IN, CNNSpec, DeviceNatureCNN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from relayrl_prototype_amd.ops import hip

    hip()  # the HIP extension must load
    return torch.device("cuda", 0)


def _two_envs(cuda, N, seed, max_steps, R):
    """An s2d-observation env and a frame-ring env with the same seed, both reset."""
    from relayrl_prototype_amd.envs.pong import DevicePong, FrameRing

    e_obs, e_ring = DevicePong(N, cuda, seed, max_steps), DevicePong(N, cuda, seed, max_steps)
    obs = torch.zeros(N, 21, 21, 64, dtype=torch.uint8, device=cuda)
    ring = FrameRing(N, R, cuda)
    fidx = torch.full((N, 4), -1, dtype=torch.int32, device=cuda)
    e_obs.reset(obs)
    e_ring.reset(ring=(ring, fidx))
    return e_obs, e_ring, obs, ring, fidx


@pytest.mark.parametrize("N,R", [(300, 5), (2048, 9)])
def test_ring_step_gives_the_rendered_observation(cuda, N, R):
    """Step + one frame into the ring == step + 4-frame render: same state, rewards, dones and,
    gathered through the frame rows, the same observation bytes -- across scoring serves and
    episode resets (max_steps 13 forces resets; the reset clamp points older frames at the reset
    frame, which the previous episode's frames in the ring must not leak into)."""
    e_obs, e_ring, obs, ring, fidx = _two_envs(cuda, N, 7, 13, R)
    torch.cuda.synchronize()
    assert torch.equal(ring.gather_s2d(fidx), obs)
    g = torch.Generator().manual_seed(4)
    resets = 0
    for _ in range(40):
        a = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
        e_obs.step(a, obs)
        e_ring.step(a, fidx, ring=ring)
        torch.cuda.synchronize()
        assert torch.equal(e_obs.state, e_ring.state)
        assert torch.equal(e_obs.rew, e_ring.rew) and torch.equal(e_obs.done, e_ring.done)
        assert torch.equal(ring.gather_s2d(fidx), obs)
        resets += int(e_obs.done.sum().item())
    assert resets > N  # every env went through at least one reset
    # P_VALID (state slot 10) follows the numpy oracle's count of distinct frames
    v = e_ring.state.view(N, -1)[:, 10]
    assert ((v >= 1) & (v <= 4)).all()


def test_ring_fill_rebuilds_the_observation_from_state(cuda):
    """pong_ring_fill (the restore path) draws the last 4 frames from the state's history alone:
    the observation it describes is the one the step kernels produced."""
    from relayrl_prototype_amd.envs.pong import FrameRing

    N = 777
    e_obs, e_ring, obs, ring, fidx = _two_envs(cuda, N, 3, 0, 7)
    g = torch.Generator().manual_seed(8)
    for _ in range(23):
        a = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
        e_obs.step(a, obs)
        e_ring.step(a, fidx, ring=ring)
    ring2 = FrameRing(N, 7, cuda)
    fidx2 = torch.full((N, 4), -1, dtype=torch.int32, device=cuda)
    # a checkpoint from before the distinct-frame count (state slot 10) existed holds 0 there: the
    # fill makes it 4, the frames it drew being the env's whole history
    e_ring.state.view(N, -1)[:, 10] = 0.0
    e_ring.ring_fill(ring2, fidx2)
    assert (e_ring.state.view(N, -1)[:, 10] == 4.0).all()
    torch.cuda.synchronize()
    assert torch.equal(ring2.gather_s2d(fidx2), obs)
    # and stepping on from the rebuilt ring stays on the observation path
    for _ in range(6):
        a = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
        e_obs.step(a, obs)
        e_ring.step(a, fidx2, ring=ring2)
        torch.cuda.synchronize()
        assert torch.equal(ring2.gather_s2d(fidx2), obs)


@pytest.mark.parametrize("N", [37, 2048])
def test_ring_fused_head_step_matches_the_obs_path(cuda, N):
    """The head + step launch writing one frame into the ring gives the obs-path launch's
    actions, log-probs, values, hidden units, state, rewards and dones, and the same observation."""
    from relayrl_prototype_amd.envs.pong import DevicePong, FrameRing

    m = DeviceNatureCNN(CNNSpec(6), cuda, max_batch=N, seed=5)
    if not (m.fc_nt and m.fused_convs):
        pytest.skip("the fused head needs the split-K fc and the fused conv stack")
    envs = [DevicePong(N, cuda, 11, 9), DevicePong(N, cuda, 11, 9)]
    obs = torch.zeros(N, 21, 21, 64, dtype=torch.uint8, device=cuda)
    ring = FrameRing(N, 9, cuda)
    fidx = [torch.zeros(N, 4, dtype=torch.int32, device=cuda) for _ in range(2)]
    envs[0].reset(obs)
    envs[1].reset(ring=(ring, fidx[0]))
    sample_t = torch.full((1,), 3, dtype=torch.int64, device=cuda)
    cur = 0
    for t in range(12):
        outs = []
        for k in range(2):
            act = torch.full((N,), -1, dtype=torch.int32, device=cuda)
            logp = torch.full((N,), float("nan"), device=cuda)
            val = torch.full((N,), float("nan"), device=cuda)
            rew = torch.full((N,), float("nan"), device=cuda)
            done = torch.full((N,), float("nan"), device=cuda)
            x = obs if k == 0 else ring.obs(fidx[cur])
            part, used, hid = m.forward_fc_partials(x, 0)
            fc_b, hp = m.head_params()
            if k == 0:
                nxt = torch.zeros_like(obs)
                envs[0].step_head(part, used, fc_b, hp, m.A, hid, act, logp, val, 123, t, sample_t, nxt, rew, done,
                                  offset=t)
            else:
                envs[1].step_head(part, used, fc_b, hp, m.A, hid, act, logp, val, 123, t, sample_t, fidx[cur ^ 1],
                                  rew, done, offset=t, ring=ring)
            torch.cuda.synchronize()
            outs.append((act.clone(), logp.clone(), val.clone(), m.hid[:N * 512].clone(), rew.clone(), done.clone(),
                         envs[k].state.clone()))
            if k == 0:
                obs = nxt
        cur ^= 1
        for a, b in zip(*outs):
            assert torch.equal(a, b)
        assert torch.equal(ring.gather_s2d(fidx[cur]), obs)


def _ring_batch(cuda, N, seed, T=5):
    """N observations as frame rows of a ring built by T + 3 env steps, and the same
    observations as s2d bytes (through the obs path)."""
    e_obs, e_ring, obs, ring, fidx = _two_envs(cuda, N, seed, 11, T + 4)
    g = torch.Generator().manual_seed(seed)
    for _ in range(T + 3):
        a = torch.randint(0, 6, (N,), dtype=torch.int32, generator=g).to(cuda)
        e_obs.step(a, obs)
        e_ring.step(a, fidx, ring=ring)
    torch.cuda.synchronize()
    return ring, fidx, obs


@pytest.mark.parametrize("N", [5, 300, 2048])
def test_ring_conv_stack_equals_the_obs_path(cuda, N):
    """The 16-wave conv stack reading its frames through the ring writes a1 / a2 / a3 bitwise
    equal to the same kernel reading the s2d observations."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    spec = CNNSpec()
    o = spec.offsets()
    params = spec.init(N).to(cuda)
    params += 0.01 * torch.randn(params.shape, generator=torch.Generator().manual_seed(N)).to(cuda)
    sh = params.bfloat16()
    ring, fidx, obs = _ring_batch(cuda, N, N)
    # a permuted batch: rows of different envs in any order (the kernel only follows fidx)
    perm = torch.randperm(N, generator=torch.Generator().manual_seed(1)).to(cuda)
    fidx, obs = fidx[perm].contiguous(), obs[perm].contiguous()
    W = [sh[o["w1"]:o["b1"]], params[o["b1"]:o["b1"] + 32], sh[o["w2"]:o["b2"]], params[o["b2"]:o["b2"] + 64],
         sh[o["w3"]:o["b3"]], params[o["b3"]:o["b3"] + 64]]
    outs = []
    # ring16: 16-byte loads on lane pairs + DPP row swap (probe 192); ring_wide: the conv1 waves load
    # whole positions of the 4 frames (probe 320)
    for form in ("s2d", "ring", "ring16", "ring_wide"):
        a1 = torch.full((N * 400 * 32,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a2 = torch.full((N * 81 * 64,), float("nan"), dtype=torch.bfloat16, device=cuda)
        a3 = torch.full((N * FC_IN,), float("nan"), dtype=torch.bfloat16, device=cuda)
        if form == "ring":
            h.conv_stack_fwd(None, *W, a1, a2, a3, N, frames=ring.frames, fidx=fidx)
        elif form == "ring16":
            h.conv_stack_fwd(None, *W, a1, a2, a3, N, probe=192, frames=ring.frames, fidx=fidx)
        elif form == "ring_wide":
            h.conv_stack_fwd(None, *W, a1, a2, a3, N, probe=320, frames=ring.frames, fidx=fidx)
        else:
            h.conv_stack_fwd(obs, *W, a1, a2, a3, N, probe=64)
        torch.cuda.synchronize()
        outs.append((a1, a2, a3))
    for other in outs[1:]:
        for f, r in zip(other, outs[0]):
            assert torch.isfinite(f.float()).all() and torch.equal(f, r)


def test_ring_conv1_wgrad_equals_the_obs_path(cuda):
    """conv1_wgrad8 reading its frames through the ring: weight and bias partials bitwise equal."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    N, grid = 1500, 256
    ring, fidx, obs = _ring_batch(cuda, N, 11)
    dy = torch.randn(N * 400 * 32, generator=torch.Generator().manual_seed(2)).bfloat16().to(cuda)
    outs = []
    for use_ring in (False, True):
        part = torch.full((2 * grid * 32 * 256,), float("nan"), device=cuda)
        bpart = torch.full((2 * grid * 32,), float("nan"), device=cuda)
        ns = h.conv1_wgrad8(None, dy, part, bpart, N, grid, frames=ring.frames, fidx=fidx) if use_ring else \
            h.conv1_wgrad8(obs, dy, part, bpart, N, grid)
        torch.cuda.synchronize()
        outs.append((part[:ns * 32 * 256], bpart[:ns * 32]))
    for f, r in zip(*outs):
        assert torch.isfinite(f).all() and torch.equal(f, r)


@pytest.mark.parametrize("E,T,grid", [(2048, 5, 256), (300, 4, 256), (37, 5, 16)])
def test_ring_conv1_wgrad_env_major_order(cuda, E, T, grid):
    """The env-major visit order (the T rows of one env back to back) sums the same products in
    another order: the reduced weight / bias gradients match the row order to fp32 reassociation,
    and every row is visited once (a row-count check through the bias of a constant dY)."""
    from relayrl_prototype_amd.ops import hip

    h = hip()
    N = E * T
    ring, fidx, _ = _ring_batch(cuda, N, 3)
    g = torch.Generator().manual_seed(5)
    dy = torch.randn(N * 400 * 32, generator=g).bfloat16().to(cuda)
    res = []
    for em in (0, T):
        part = torch.full((2 * grid * 32 * 256,), float("nan"), device=cuda)
        bpart = torch.full((2 * grid * 32,), float("nan"), device=cuda)
        ns = h.conv1_wgrad8(None, dy, part, bpart, N, grid, frames=ring.frames, fidx=fidx, env_major_T=em)
        torch.cuda.synchronize()
        res.append((part[:ns * 32 * 256].view(ns, -1).double().sum(0), bpart[:ns * 32].view(ns, -1).double().sum(0)))
    (w0, b0), (w1, b1) = res
    torch.testing.assert_close(w1, w0, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(b1, b0, rtol=1e-5, atol=1e-4)
    ones = torch.ones(N * 400 * 32, dtype=torch.bfloat16, device=cuda)
    part = torch.zeros(2 * grid * 32 * 256, device=cuda)
    bpart = torch.zeros(2 * grid * 32, device=cuda)
    ns = h.conv1_wgrad8(None, ones, part, bpart, N, grid, frames=ring.frames, fidx=fidx, env_major_T=T)
    torch.cuda.synchronize()
    assert torch.equal(bpart[:ns * 32].view(ns, 32).sum(0).cpu(), torch.full((32,), float(N * 400)))


@pytest.mark.parametrize("fused_head", ["1", "0"])
def test_pixel_update_frame_ring_matches_the_obs_path(cuda, monkeypatch, fused_head):
    """A2C on the frame ring trains the same trajectory bitwise as on 4-frame observations
    (captured graphs, both buffer parities, the 16-wave forward), with the policy head inside the
    step launch and without it; a checkpoint of the ring trainer restores its observation."""
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    monkeypatch.setenv("RRL_CNN_FWD_LAYOUT", "64")
    monkeypatch.setenv("RRL_PONG_FUSED_HEAD", fused_head)
    monkeypatch.setenv("RRL_CNN_WGRAD1_ENV_MAJOR", "0")  # the row order: bitwise the obs path
    runs = []
    for ring in (False, True):
        tr = PixelA2CTrainer(PixelA2CConfig(num_envs=300, rollout_len=4, seed=6, use_graphs=True, max_episode_steps=7,
                                            frame_ring=ring, fused_render=False), device=cuda)
        assert (tr.ring is not None) == ring and tr.fused_head == (fused_head == "1")
        for _ in range(5):
            tr.train_epoch()
        torch.cuda.synchronize()
        runs.append(tr)
    a, b = runs
    assert a._graph is not None and b._graph is not None
    assert torch.equal(a.act, b.act) and torch.equal(a.rew, b.rew) and torch.equal(a.done, b.done)
    assert torch.equal(b.ring.gather_s2d(b.obs[0]), a.obs[0])
    torch.testing.assert_close(b.model.params, a.model.params, rtol=0, atol=0)
    assert a.metrics()["Episodes"] == b.metrics()["Episodes"] > 0
    # checkpoint round trip: the restored ring trainer's observation is rebuilt from the env state
    st = b.state_dict()
    c = PixelA2CTrainer(PixelA2CConfig(num_envs=300, rollout_len=4, seed=6, use_graphs=True, max_episode_steps=7,
                                       frame_ring=True, fused_render=False), device=cuda)
    c.load_state_dict(st)
    torch.cuda.synchronize()
    assert torch.equal(c.ring.gather_s2d(c.obs[0]), a.obs[0])
    a.train_epoch()
    c.train_epoch()
    torch.cuda.synchronize()
    torch.testing.assert_close(c.model.params, a.model.params, rtol=0, atol=0)


def test_pixel_update_frame_ring_env_major_wgrad(cuda, monkeypatch):
    """The shipped ring update (conv1 weight gradient env-major) differs from the row order only by
    fp32 reassociation of dW1: one update from the same state gives the same gradients to 1e-4."""
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    monkeypatch.setenv("RRL_CNN_FWD_LAYOUT", "64")
    grads = []
    for em in ("0", "1"):
        monkeypatch.setenv("RRL_CNN_WGRAD1_ENV_MAJOR", em)
        tr = PixelA2CTrainer(PixelA2CConfig(num_envs=512, rollout_len=5, seed=2, use_graphs=False, frame_ring=True,
                                            fused_render=False), device=cuda)
        tr.train_epoch()
        torch.cuda.synchronize()
        grads.append(tr.model.grad.clone())
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-4, atol=1e-6)


def test_pong_ring_data_parallel_two_gloo_ranks_shared_gpu(cuda):
    """Two ranks of the Pong A2C bench (frame ring on) on one GPU over gloo: the all-reduced
    updates leave bitwise the same parameters on both ranks."""
    import json
    import os
    import socket
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RRL_DIST_BACKEND="gloo", RRL_FORCE_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={port}", "benchmarks/pong_a2c_bench.py", "--gpus", "2", "--num-envs", "128", "--steps", "3",
           "--warmup", "1"]
    r = subprocess.run(cmd, cwd=repo, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["frame_ring"] is True and rec["params_in_sync"] is True and rec["value"] > 0


def test_ring_elastic_snapshot_restore_replays_the_epochs(cuda):
    """The elastic epoch-start snapshot (launcher.EpochSnapshot) leaves the ring's frames out and
    the restore rebuilds them from the env state (set_counters -> pong_ring_fill): two epochs
    replayed after a restore -- over a frame store scribbled in between -- are bitwise the two
    epochs that followed the snapshot."""
    from relayrl_prototype_amd.runtime.launcher import EpochSnapshot
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    tr = PixelA2CTrainer(PixelA2CConfig(num_envs=300, rollout_len=4, seed=3, use_graphs=True, max_episode_steps=7,
                                        frame_ring=True, fused_render=False), device=cuda)
    for _ in range(3):  # eager warm-up, capture + replay of both buffer parities
        tr.train_epoch()
    snap = EpochSnapshot()
    snap.take(tr)
    assert all(t.data_ptr() != tr.ring.frames.data_ptr() for t in tr.snapshot_tensors())
    runs = []
    for _ in range(2):
        for _ in range(2):
            tr.train_epoch()
        torch.cuda.synchronize()
        runs.append((tr.model.params.clone(), tr.act.clone(), tr.rew.clone()))
        tr.ring.frames.fill_(7)  # whatever the store held is gone
        snap.restore(tr)
    for a, b in zip(*runs):
        assert torch.equal(a, b)
