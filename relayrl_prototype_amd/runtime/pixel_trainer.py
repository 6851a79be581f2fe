"""A2C on pixels: PongSynth-v0 + Nature-CNN actor-critic (BASELINE.json config 4:
"Actor-critic (A2C) Atari Pong pixels -- CNN encoder on MFMA, 8-GPU DP grad all-reduce").

One update on each rank (one process per GPU), everything device resident:

  1. rollout: T steps x N envs -- conv stack + fc on MFMA, fused policy/value head with
     Philox sampling, Pong physics + 4-frame render straight into the uint8 obs ring;
     the forward activations are KEPT (params do not change inside a rollout), so the
     update needs no second forward pass
  2. bootstrap value of obs[T], n-step returns via the GAE scan with lambda = 1
  3. fused A2C head backward -> fc / conv weight gradients (transposed-LDS MFMA GEMMs,
     split-K partials), data gradients + col2im with the ReLU mask fused
  4. DP: RCCL all-reduce of the flat fp32 gradient in two buckets, the fc+head bucket
     overlapped with the conv backward (world > 1)
  5. global-norm clip + Adam + bf16 shadow weights in one kernel

The whole update (~50 launches, plus the two bucketed RCCL all-reduces at world > 1) is
captured into a hipGraph after one eager warm-up update and replayed: RNG step counters and
the Adam step live on the device, so replays draw fresh samples and bias corrections without
host involvement.  With several ranks the capture needs RCCL (``Comm.graph_safe``); the
all-reduces then replay inside the graph on every rank.

The CPU path (tests, no GPU) runs the same algorithm through the PyTorch oracle model
and the numpy Pong reference.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Optional

import torch

from ..models.nature_cnn import CNNSpec, DeviceNatureCNN, a2c_loss, reference_forward
from ..parallel.comm import Comm
from ..utils.tracing import PhaseTimer, gc_paused


@dataclass
class PixelA2CConfig:
    env: str = "PongSynth-v0"
    num_envs: int = 512            # envs per rank
    rollout_len: int = 5           # A2C n-step
    gamma: float = 0.99
    lr: float = 2.5e-4
    vf_coef: float = 0.5
    ent_coef: float = 0.01
    max_grad_norm: float = 0.5
    seed: int = 0
    max_episode_steps: int = 27000 // 4
    phase_timing: bool = False
    use_graphs: bool = True        # capture the whole update (with its RCCL all-reduces) as one hipGraph
    # GPU: the conv kernels draw the observations themselves from 16-float frame histories (no
    # [T+1, N, 21, 21, 64] observation tensor is written or read); None = RRL_PONG_FUSED_RENDER
    fused_render: Optional[bool] = None
    # GPU: each env step renders ONE new frame into a frame ring (envs/pong.FrameRing) and an
    # observation is 4 frame rows; the conv kernels interleave the frames as they load them (7 KB
    # instead of 28 KB written per env step: step launch 24.9 -> 19.4 us, update 1186.7 ->
    # 1166.6 us at 2,048 envs, ABBA +0.4 % / +1.0 % at 2,048 / 8,192 envs,
    # profiles/r6_pong_ring_v3_ab.txt).  None = RRL_PONG_FRAME_RING (default on)
    frame_ring: Optional[bool] = None

    def to_dict(self):
        return asdict(self)


class PixelA2CTrainer:
    def __init__(self, cfg: PixelA2CConfig, comm: Optional[Comm] = None, device=None):
        if cfg.env != "PongSynth-v0":
            raise ValueError(f"pixel trainer supports PongSynth-v0, not {cfg.env!r}")
        self.cfg = cfg
        self.comm = comm or Comm()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.on_gpu = self.device.type == "cuda"
        self.spec = CNNSpec(act_dim=6)
        N, T = cfg.num_envs, cfg.rollout_len
        rank = self.comm.rank
        env_seed = (cfg.seed * 1000003 + rank * 7919 + 17) & 0x7FFFFFFFFFFFFFFF
        self.sample_seed = (cfg.seed * 2654435761 + rank * 97 + 5) & 0x7FFFFFFFFFFFFFFF
        dev = self.device
        import os

        if cfg.fused_render is None:
            cfg.fused_render = os.environ.get("RRL_PONG_FUSED_RENDER", "0") == "1"
        self.fused_render = bool(cfg.fused_render) and self.on_gpu
        if cfg.frame_ring is None:
            cfg.frame_ring = os.environ.get("RRL_PONG_FRAME_RING", "1") == "1"
        self.ring = None
        if self.fused_render:  # the frame histories the conv kernels render from
            self.obs = torch.zeros((T + 1, N, 16), dtype=torch.float32, device=dev)
        elif cfg.frame_ring and self.on_gpu and os.environ.get("RRL_CNN_FUSED", "1") != "0" and \
                int(os.environ.get("RRL_CNN_FWD_LAYOUT", "0")) in (0, 64):  # the 16-wave conv stack reads the ring
            from ..envs.pong import FrameRing

            # T + 4 slots: a rollout's observations read the frames of steps t0 - 3 .. t0 + T
            self.ring = FrameRing(N, T + 4, dev)
            self.obs = torch.zeros((T + 1, N, 4), dtype=torch.int32, device=dev)  # frame rows per observation
        else:
            self.obs = torch.zeros((T + 1, N, 21, 21, 64), dtype=torch.uint8, device=dev)  # space-to-depth frames
        # GPU: two observation buffers used alternately -- update k rolls out of buffer k % 2 and
        # renders its last observation straight into slot 0 of the other one, where update k + 1
        # starts (no obs[T] -> obs[0] copy of 58 MB per update); one captured graph per buffer
        two = dev.type == "cuda" and os.environ.get("RRL_PONG_OBS_COPY", "0") != "1"  # 1: the copy path (A/B)
        self._obs_bufs = [self.obs, torch.zeros_like(self.obs)] if two else [self.obs]
        self._par = 0
        self.act = torch.zeros((T, N), dtype=torch.int32, device=dev)
        self.logp = torch.zeros((T, N), device=dev)
        self.val = torch.zeros((T + 1, N), device=dev)
        self.rew = torch.zeros((T, N), device=dev)
        self.done = torch.zeros((T, N), device=dev)
        self.ep_sum = torch.zeros(4, dtype=torch.float64, device=dev)  # n, sum ret, sum len, sum ret^2
        self.total_steps = 0
        self.updates = 0
        self.timer = PhaseTimer(dev if cfg.phase_timing and self.on_gpu else None, enabled=cfg.phase_timing)
        if self.on_gpu:
            from ..envs.pong import DevicePong

            self.model = DeviceNatureCNN(self.spec, dev, max_batch=N * (T + 1), seed=cfg.seed)
            assert self.ring is None or (self.model.fused_convs and self.model.fwd_layout in (0, 64))
            self.env = DevicePong(N, dev, env_seed, cfg.max_episode_steps)
            # the rollout's policy head inside the env-step launch: +1.6 % at 2,048 envs, -0.3 % at
            # 8,192 (profiles/r5_pong_fused_head_ab.jsonl), so on up to 4,096 envs by default;
            # RRL_PONG_FUSED_HEAD=1 / 0 forces it on / off
            fh = os.environ.get("RRL_PONG_FUSED_HEAD", "")
            self.fused_head = ((fh == "1") if fh else N <= 4096) and not self.fused_render and \
                self.model.fc_nt and self.model.A <= 8
            if self.fused_render:
                self.env.reset(hist_out=self.obs[0])
            elif self.ring is not None:
                self.env.reset(ring=(self.ring, self.obs[0]))
            else:
                self.env.reset(self.obs[0])
            self.sample_t = torch.zeros(1, dtype=torch.int64, device=dev)  # Philox step of the action sampler
            self.adv = torch.zeros(T, N, device=dev)
            self.ret = torch.zeros(T, N, device=dev)
            from ..ops import hip

            self._stats_part = torch.zeros(int(hip().scan_tm_parts(N)), 3, device=dev)
            self._graph = None  # the graph of the current buffer parity (None before capture)
            self._graphs = {}
            self._warm = False
        else:
            from ..envs.pong import PongRef

            self.params = self.spec.init(cfg.seed).requires_grad_(True)
            self.opt = torch.optim.Adam([self.params], lr=cfg.lr, eps=1e-5)
            self.env = PongRef(N, env_seed, cfg.max_episode_steps)
            self.obs[0] = torch.from_numpy(self.env.reset())
            self.gen = torch.Generator().manual_seed(self.sample_seed)
        self.comm.barrier() if self.comm.multi else None

    # ------------------------------------------------------------------ GPU
    def _ob(self, rows):
        """Observations for the model: the s2d / history rows themselves, or frame rows of the ring."""
        return rows if self.ring is None else self.ring.obs(rows)

    def _rollout_gpu(self, base, nxt):
        cfg, m, N, T = self.cfg, self.model, self.cfg.num_envs, self.cfg.rollout_len
        ring = self.ring
        m.begin_update()  # the transposed Wfc refresh beside the rollout (side stream)
        for t in range(T):
            # the last observation goes straight to the next update's start slot
            out = base[t + 1] if (t + 1 < T or nxt is None) else nxt[0]
            if self.fused_head:  # conv stack + fc partials, then head + env step + render in one launch
                part, used, hid = m.forward_fc_partials(self._ob(base[t]), t * N)
                fc_b, hp = m.head_params()
                self.env.step_head(part, used, fc_b, hp, m.A, hid, self.act[t], self.logp[t], self.val[t],
                                   self.sample_seed, t, self.sample_t, out, self.rew[t], self.done[t], offset=t,
                                   ring=ring)
                continue
            m.act(self._ob(base[t]), t * N, self.act[t], self.logp[t], self.val[t], self.sample_seed, t,
                  step_base=self.sample_t)
            if self.fused_render:
                self.env.step(self.act[t], None, self.rew[t], self.done[t], offset=t, hist_out=out)
            else:
                self.env.step(self.act[t], out, self.rew[t], self.done[t], offset=t, ring=ring)
        # the sampling, env and Adam step counters advance inside the update's scan launch
        # (_update_gpu; every rollout is followed by one update)
        # bootstrap V(obs[T]) with the pre-update weights; its activations go to the
        # scratch rows [T*N, (T+1)*N) so the stored rollout activations stay intact
        m.value(self._ob(base[T] if nxt is None else nxt[0]), cfg.rollout_len * N, self.val[cfg.rollout_len])

    def _update_gpu(self, base):
        from ..ops import gae_scan_tm

        cfg, m = self.cfg, self.model
        N, T = cfg.num_envs, cfg.rollout_len
        B = N * T
        with self.timer.phase("Returns"):
            # + the sampling / env / Adam step counters of this rollout and update (the Adam step of
            # apply(step_bumped=True) below): no launch of their own
            adv, ret, _ = gae_scan_tm(self.rew, self.done, self.val, cfg.gamma, 1.0, self.adv, self.ret,
                                      self._stats_part, stats=False,
                                      counters=((self.sample_t, T), (self.env.step_t, T), (m.step_t, 1)))
        with self.timer.phase("Backward"):
            if self.ring is not None:
                x = self.ring.obs(base[:T].reshape(B, 4), rollout_len=T)
            else:
                x = base[:T].reshape(B, 16) if self.fused_render else base[:T].reshape(B, 21, 21, 64)
            stats = m.backward(x, self.act.reshape(B), adv.reshape(B),
                               ret.reshape(B), cfg.vf_coef, cfg.ent_coef, comm=self.comm)
        with self.timer.phase("Optimize"):
            m.apply(cfg.lr, cfg.max_grad_norm, self.comm, step_bumped=True)
        return stats

    # ------------------------------------------------------------------ CPU
    def _rollout_cpu(self):
        cfg, N = self.cfg, self.cfg.num_envs
        with torch.no_grad():
            for t in range(cfg.rollout_len):
                logits, value, _ = reference_forward(self.spec, self.params, self.obs[t])
                a = torch.multinomial(torch.softmax(logits, -1), 1, generator=self.gen)[:, 0]
                self.act[t] = a.int()
                self.val[t] = value
                r, d, fr, fl = self.env.step(a.numpy())
                self.rew[t] = torch.from_numpy(r)
                self.done[t] = torch.from_numpy(d)
                self.obs[t + 1] = torch.from_numpy(self.env.render())
                self.ep_sum += torch.tensor([d.sum(), (fr * d).sum(), (fl * d).sum(), (fr * fr * d).sum()],
                                            dtype=torch.float64)

    def _update_cpu(self):
        from ..ops import gae_scan_tm

        cfg = self.cfg
        N, T = cfg.num_envs, cfg.rollout_len
        B = N * T
        adv, ret, _ = gae_scan_tm(self.rew, self.done, self.val, cfg.gamma, 1.0)
        logits, value, _ = reference_forward(self.spec, self.params, self.obs[:T].reshape(B, 21, 21, 64))
        loss, pg, vf, ent = a2c_loss(logits, value, self.act.reshape(B), adv.reshape(B), ret.reshape(B), cfg.vf_coef,
                                     cfg.ent_coef)
        self.opt.zero_grad()
        loss.backward()
        if self.comm.multi:
            self.comm.all_reduce_sum_(self.params.grad)
            self.params.grad.mul_(1.0 / self.comm.world)
        torch.nn.utils.clip_grad_norm_([self.params], cfg.max_grad_norm)
        self.opt.step()
        return torch.tensor([[pg.item() * B, vf.item() * B, ent.item() * B, float(B)]])

    # ------------------------------------------------------------------ API
    def _gpu_update_body(self, par: int):
        base = self._obs_bufs[par]
        nxt = self._obs_bufs[par ^ 1] if len(self._obs_bufs) == 2 else None
        with self.timer.phase("Rollout"):
            self._rollout_gpu(base, nxt)
        stats = self._update_gpu(base)
        if nxt is None:
            base[0].copy_(base[self.cfg.rollout_len])
        return stats

    def _graphable(self) -> bool:
        # world > 1: the bucketed RCCL all-reduces are captured with the rest of the update
        return self.on_gpu and self.cfg.use_graphs and self.comm.graph_safe and not self.timer.enabled

    def train_epoch(self):
        cfg = self.cfg
        N, T = cfg.num_envs, cfg.rollout_len
        if self.on_gpu:
            par = self._par
            if self._graphable() and par in self._graphs:
                g, stats = self._graphs[par]
                # (replayed on a high-priority stream instead: -52 % at 2,048 envs, -30 % at 8,192,
                # profiles/r5_pong_side_early_main_ab.txt)
                g.replay()
            elif self._graphable() and self._warm:
                # capture once per buffer parity (kernel attributes / workspaces were set up by the
                # eager warm-up)
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    # thread_local: HIP calls of other threads (a server's transport / relay
                    # threads) neither fail nor invalidate this capture
                    with gc_paused(), torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                        stats = self._gpu_update_body(par)
                torch.cuda.current_stream().wait_stream(s)
                self._graphs[par] = (g, stats)
                g.replay()  # the capture itself does not execute
            else:
                stats = self._gpu_update_body(par)
                self._warm = True
            self._graph = self._graphs.get(par, (None,))[0]
            self._par = (self._par + 1) % len(self._obs_bufs)
            self.obs = self._obs_bufs[self._par]
        else:
            with self.timer.phase("Rollout"):
                self._rollout_cpu()
            with torch.no_grad():
                _, v, _ = reference_forward(self.spec, self.params, self.obs[T])
            self.val[T] = v
            stats = self._update_cpu()
            self.obs[0].copy_(self.obs[T])
        self.total_steps += N * T
        self.updates += 1
        self._last_stats = stats
        return stats

    def metrics(self):
        s = (self.env.episode_stats() if self.on_gpu else self.ep_sum).tolist()
        st = self._last_stats.sum(0).tolist() if hasattr(self, "_last_stats") else [0, 0, 0, 1]
        cnt = max(st[3], 1.0)
        n = s[0]
        out = {"Updates": self.updates, "EnvSteps": self.total_steps * self.comm.world,
               "Episodes": n, "AverageEpRet": s[1] / n if n else float("nan"),
               "EpLen": s[2] / n if n else float("nan"), "LossPi": st[0] / cnt, "LossV": st[1] / cnt,
               "Entropy": st[2] / cnt}
        return out

    # elastic epoch-start snapshot (launcher.EpochSnapshot): device tensors + host counters
    def snapshot_tensors(self):
        if not self.on_gpu:
            ts = [self.params.data]
            for st in self.opt.state.values():
                ts += [v for v in st.values() if torch.is_tensor(v)]
            return ts
        m = self.model
        # (the frame ring's frames are not snapshotted -- up to 520 MB per epoch at 8,192 envs: the
        # restore rebuilds them from the env state, set_counters)
        return [m.params, m.m, m.v, m.step_t, self.env.state, self.env.step_t, self.env.ep_acc, self.sample_t,
                self.obs[0]]

    def counters(self) -> dict:
        return {"updates": self.updates, "total_steps": self.total_steps}

    def set_counters(self, c: dict):
        """After an elastic snapshot restore (launcher.EpochSnapshot): host counters, the bf16
        shadow weights and -- frame ring -- the ring's frames and the current observation's rows,
        rebuilt from the restored env state."""
        self.updates, self.total_steps = int(c["updates"]), int(c["total_steps"])
        if self.on_gpu:
            self.model.refresh_shadow()
            if self.ring is not None:
                self.env.ring_fill(self.ring, self.obs[0])

    def drop_graphs(self):
        if self.on_gpu:
            self._graphs.clear()
            self._graph = None

    def state_dict(self) -> dict:
        st = {"updates": self.updates, "total_steps": self.total_steps, "obs0": self.obs[0].cpu(),
              "cfg": self.cfg.to_dict()}
        if self.on_gpu:
            st["model"] = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
            st["env_state"] = self.env.state.cpu()
            st["env_step"] = self.env.step_count
            st["sample_step"] = int(self.sample_t.item())
        else:
            st["params"] = self.params.detach().cpu()
            st["opt"] = self.opt.state_dict()
        return st

    def load_state_dict(self, st: dict):
        self.updates = int(st["updates"])
        self.total_steps = int(st["total_steps"])
        obs0 = st["obs0"]
        if obs0.shape == self.obs[0].shape and obs0.dtype == self.obs.dtype:
            self.obs[0].copy_(obs0.to(self.device))
        if self.on_gpu:
            self.model.load_state_dict({k: v.to(self.device) for k, v in st["model"].items()})
            self.env.state.copy_(st["env_state"].to(self.device))
            self.env.step_count = int(st["env_step"])
            self.sample_t.fill_(int(st.get("sample_step", self.updates * self.cfg.rollout_len)))
            # the observation is a function of the env state: rebuilt when the checkpoint's
            # observation form differs (s2d vs frame ring), and always for the ring (its frames
            # are not in the checkpoint)
            if self.ring is not None:
                self.env.ring_fill(self.ring, self.obs[0])
            elif obs0.shape != self.obs[0].shape or obs0.dtype != self.obs.dtype:
                if self.fused_render:
                    self.obs[0].copy_(self.env.state.view(self.cfg.num_envs, -1)[:, 16:32])
                else:
                    self.env.h.pong_render(self.env.state, self.obs[0], self.cfg.num_envs)
        else:
            with torch.no_grad():
                self.params.copy_(st["params"])
            self.opt.load_state_dict(st["opt"])

    def sync_from_rank0(self, src: int = 0):
        """Rank ``src``'s model and optimiser state everywhere (elastic re-form / auto-resume)."""
        if not self.comm.multi:
            return
        if self.on_gpu:
            m = self.model
            for t in (m.params, m.m, m.v, m.step_t):
                self.comm.broadcast_(t, src)
            m.refresh_shadow()
        else:
            with torch.no_grad():
                self.comm.broadcast_(self.params.data, src)
            for st in self.opt.state.values():
                for v in st.values():
                    if torch.is_tensor(v):
                        self.comm.broadcast_(v, src)

    def episode_sums(self) -> tuple:
        """(finished episodes, sum of their returns) since the previous call, global over
        ranks: the windowed threshold check (vec_trainer.SolvedCheck) needs the newest
        episodes, not metrics()' running mean since the start.  One synchronising read."""
        tot = (self.env.episode_stats() if self.on_gpu else self.ep_sum.clone())[:2].double()
        if self.comm.multi:
            tot = tot if (self.comm.backend == "nccl" or not tot.is_cuda) else tot.cpu()
            self.comm.all_reduce_sum_(tot)
        n, s = tot.tolist()
        n0, s0 = getattr(self, "_sums_seen", (0.0, 0.0))
        self._sums_seen = (n, s)
        return n - n0, s - s0

    def reset_episode_stats(self):
        self.ep_sum.zero_()
        self._sums_seen = (0.0, 0.0)
        if self.on_gpu:
            self.env.ep_acc.zero_()
