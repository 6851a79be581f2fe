"""PongSynth-v0 -- device Pong with Atari-style observations (csrc/kernels/pong.hip).

``PongRef`` is the vectorised numpy oracle of the kernel (same state layout, same
float32 arithmetic order, same Philox draws), used by the CPU trainer path and by the
GPU numerics tests; ``DevicePong`` drives the kernels on a torch device.

Interface (Atari Pong): 6 actions (0 NOOP, 1 FIRE, 2 RIGHT = up, 3 LEFT = down,
4 RIGHTFIRE, 5 LEFTFIRE), frame-skip 4, 84x84 grayscale frames, the 4 most recent
frames stacked (oldest first), reward +1 / -1 per point, episode over at 21 points (or
``max_steps`` agent steps).

Observation layout: uint8 [21, 21, 64] = space-to-depth(4) of the NHWC [84, 84, 4]
stack, obs[a][b][dy*16 + dx*4 + f] = frame f at pixel (4a + dy, 4b + dx); convert with
``s2d_to_nhwc`` / ``nhwc_to_s2d``.  The layout is what the first conv layer streams
(an 8x8/4 conv == a 2x2/1 conv over 64 contiguous channels).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.philox import philox4x32, u01

NUM_ACTIONS = 6
OBS_SHAPE = (21, 21, 64)
NHWC_SHAPE = (84, 84, 4)
STATE = 32
HW = 84
BX, BY, VX, VY, PA, PO, SA, SO, T, RET, VALID = range(11)  # VALID: distinct frames in the stack (1..4)
HIST = 16
TOP, BOT, PAD_HALF, BALL = 2.0, 82.0, 5.0, 2.0
AGENT_X, OPP_X, PAD_W = 76.0, 6.0, 2.0
PAD_SPEED, OPP_SPEED, MAX_VY, MAX_VX = 2.5, 1.6, 3.0, 3.0

f32 = np.float32


def _rand(seed, step, rows, tag):
    k0, k1 = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
    return philox4x32(rows.astype(np.uint32), np.full_like(rows, step & 0xFFFFFFFF, dtype=np.uint32),
                      np.full_like(rows, (step >> 32) & 0xFFFFFFFF, dtype=np.uint32),
                      np.full_like(rows, tag, dtype=np.uint32), k0, k1)


def nhwc_to_s2d(x):
    """[..., 84, 84, 4] -> [..., 21, 21, 64] (numpy or torch)."""
    lead = x.shape[:-3]
    y = x.reshape(*lead, 21, 4, 21, 4, 4)
    n = len(lead)
    perm = tuple(range(n)) + (n, n + 2, n + 1, n + 3, n + 4)
    y = y.transpose(perm) if isinstance(y, np.ndarray) else y.permute(perm)
    return y.reshape(*lead, 21, 21, 64)


def s2d_to_nhwc(x):
    """[..., 21, 21, 64] -> [..., 84, 84, 4] (numpy or torch)."""
    lead = x.shape[:-3]
    y = x.reshape(*lead, 21, 21, 4, 4, 4)
    n = len(lead)
    perm = tuple(range(n)) + (n, n + 2, n + 1, n + 3, n + 4)
    y = y.transpose(perm) if isinstance(y, np.ndarray) else y.permute(perm)
    return y.reshape(*lead, 84, 84, 4)


class PongRef:
    def __init__(self, num_envs: int, seed: int = 0, max_steps: int = 27000 // 4):
        self.N = int(num_envs)
        self.seed = int(seed)
        self.max_steps = int(max_steps)
        self.s = np.zeros((self.N, STATE), f32)
        self.step_count = 0

    # --- pieces shared with the kernel
    def _serve(self, s, idx, r):
        s[idx, BX] = f32(41.0)
        s[idx, BY] = f32(30.0) + f32(24.0) * u01(r[0][idx])
        s[idx, VX] = np.where(r[1][idx] & 1, f32(1.5), f32(-1.5))
        s[idx, VY] = (u01(r[2][idx]) - f32(0.5)) * f32(3.0)

    @staticmethod
    def _push_hist(s, idx):
        h = s[idx, HIST:HIST + 16].reshape(-1, 4, 4)
        h[:, :3] = h[:, 1:].copy()
        h[:, 3] = s[idx][:, [BX, BY, PA, PO]]
        s[idx, HIST:HIST + 16] = h.reshape(-1, 16)

    def _reset(self, s, idx, r):
        s[idx] = 0
        s[idx, PA] = 42.0
        s[idx, PO] = 42.0
        self._serve(s, idx, r)
        for _ in range(4):
            self._push_hist(s, idx)
        s[idx, VALID] = 1.0

    def reset(self):
        rows = np.arange(self.N, dtype=np.uint32)
        r = _rand(self.seed, self.step_count, rows, 0x51)
        self._reset(self.s, np.arange(self.N), r)
        self.step_count += 1
        return self.render()

    def step(self, act):
        s = self.s
        N = self.N
        rows = np.arange(N, dtype=np.uint32)
        r0 = _rand(self.seed, self.step_count, rows, 0x51)
        a = np.asarray(act).reshape(N)
        d = np.where((a == 2) | (a == 4), f32(-1), np.where((a == 3) | (a == 5), f32(1), f32(0))).astype(f32)
        reward = np.zeros(N, f32)
        point = np.zeros(N, bool)
        for _ in range(4):
            live = ~point
            pa = np.clip(s[:, PA] + d * f32(PAD_SPEED), f32(TOP + PAD_HALF), f32(BOT - PAD_HALF))
            s[:, PA] = np.where(live, pa, s[:, PA])
            target = np.where(s[:, VX] < 0, s[:, BY] + f32(1), f32(42))
            dd = np.clip(target - s[:, PO], f32(-OPP_SPEED), f32(OPP_SPEED))
            po = np.clip(s[:, PO] + dd, f32(TOP + PAD_HALF), f32(BOT - PAD_HALF))
            s[:, PO] = np.where(live, po, s[:, PO])
            bx = s[:, BX] + s[:, VX]
            by = s[:, BY] + s[:, VY]
            vy = s[:, VY].copy()
            lo = by < f32(TOP)
            by = np.where(lo, f32(2 * TOP) - by, by)
            vy = np.where(lo, -vy, vy)
            hi = by + f32(BALL) > f32(BOT)
            by = np.where(hi, f32(2 * (BOT - BALL)) - by, by)
            vy = np.where(hi, -vy, vy)
            cy = by + f32(0.5 * BALL)
            vx = s[:, VX].copy()
            hit_a = (vx > 0) & (bx + f32(BALL) >= f32(AGENT_X)) & (s[:, BX] + f32(BALL) <= f32(AGENT_X + PAD_W)) & \
                (np.abs(cy - s[:, PA]) <= f32(PAD_HALF + 1))
            hit_o = ~hit_a & (vx < 0) & (bx <= f32(OPP_X + PAD_W)) & (s[:, BX] >= f32(OPP_X)) & \
                (np.abs(cy - s[:, PO]) <= f32(PAD_HALF + 1))
            bx = np.where(hit_a, f32(AGENT_X - BALL), np.where(hit_o, f32(OPP_X + PAD_W), bx))
            spd = np.minimum(np.abs(vx) * f32(1.05), f32(MAX_VX))
            vy_a = np.clip(vy + f32(0.35) * (cy - s[:, PA]), f32(-MAX_VY), f32(MAX_VY))
            vy_o = np.clip(vy + f32(0.35) * (cy - s[:, PO]), f32(-MAX_VY), f32(MAX_VY))
            new_vx = np.where(hit_a, -spd, np.where(hit_o, spd, vx))
            new_vy = np.where(hit_a, vy_a, np.where(hit_o, vy_o, vy))
            s[:, BX] = np.where(live, bx, s[:, BX])
            s[:, BY] = np.where(live, by, s[:, BY])
            s[:, VX] = np.where(live, new_vx, s[:, VX])
            s[:, VY] = np.where(live, new_vy, s[:, VY])
            opp = live & (bx > f32(HW))
            ag = live & ~opp & (bx + f32(BALL) < f32(0))
            reward = reward - opp.astype(f32) + ag.astype(f32)
            s[:, SO] += opp
            s[:, SA] += ag
            point |= opp | ag
        if point.any():
            self._serve(s, np.flatnonzero(point), r0)
        s[:, T] += 1
        s[:, RET] += reward
        self._push_hist(s, np.arange(N))
        s[:, VALID] = np.minimum(s[:, VALID] + f32(1), f32(4))
        over = (s[:, SA] >= 21) | (s[:, SO] >= 21) | ((self.max_steps > 0) & (s[:, T] >= self.max_steps))
        fin_ret = np.where(over, s[:, RET], 0).astype(f32)
        fin_len = np.where(over, s[:, T], 0).astype(f32)
        if over.any():
            r1 = _rand(self.seed, self.step_count, rows, 0x52)
            self._reset(s, np.flatnonzero(over), r1)
        self.step_count += 1
        return reward, over.astype(f32), fin_ret, fin_len

    def render(self) -> np.ndarray:
        """Observation in the device layout (space-to-depth, [N, 21, 21, 64])."""
        return np.ascontiguousarray(nhwc_to_s2d(self.render_nhwc()))

    def render_nhwc(self) -> np.ndarray:
        N = self.N
        h = self.s[:, HIST:HIST + 16].reshape(N, 4, 4)
        fy = np.arange(HW, dtype=f32) + f32(0.5)
        fx = fy
        wall = (fy < TOP) | (fy >= BOT)
        obs = np.where(wall[None, :, None, None], np.uint8(100), np.uint8(0)).astype(np.uint8)
        obs = np.broadcast_to(obs, (N, HW, HW, 4)).copy()
        for f in range(4):
            bx, by, pa, po = h[:, f, 0], h[:, f, 1], h[:, f, 2], h[:, f, 3]
            rows_pa = np.abs(fy[None] - pa[:, None]) < PAD_HALF
            rows_po = np.abs(fy[None] - po[:, None]) < PAD_HALF
            rows_b = (fy[None] >= by[:, None]) & (fy[None] < by[:, None] + BALL)
            cols_a = (fx >= AGENT_X) & (fx < AGENT_X + PAD_W)
            cols_o = (fx >= OPP_X) & (fx < OPP_X + PAD_W)
            cols_b = (fx[None] >= bx[:, None]) & (fx[None] < bx[:, None] + BALL)
            m = (rows_pa[:, :, None] & cols_a[None, None, :]) | (rows_po[:, :, None] & cols_o[None, None, :]) | \
                (rows_b[:, :, None] & cols_b[:, None, :])
            obs[..., f] = np.where(m, np.uint8(255), obs[..., f])
        return obs


FRAME_BYTES = 7056  # one 84 x 84 frame in s2d order [21][21][4][4] (pong_render.h)


class FrameRing:
    """The frame store of the frame-ring observation path (csrc/kernels/pong_render.h): ``R``
    slots of one frame per env, ``frames`` [R, N, 7056] uint8.  Each env step renders ONE new
    frame (slot ``step mod R``); an observation is the int32 row [4] of its frames' store rows
    (``slot * N + env``, oldest first).  ``R >= T + 4`` keeps every frame of a rollout's
    observations (steps t0 - 3 .. t0 + T) alive until the update has read them."""

    def __init__(self, num_envs: int, slots: int, device):
        if slots < 5:
            raise ValueError("a frame ring needs >= 5 slots (rollout_len + 4)")
        self.N, self.R = int(num_envs), int(slots)
        self.frames = torch.zeros(self.R * self.N * FRAME_BYTES, dtype=torch.uint8, device=device)

    def obs(self, fidx: torch.Tensor, rollout_len: int = 0) -> "FrameRingObs":
        """Observations of frame rows ``fidx``; ``rollout_len`` T > 1 marks them as a T-step
        rollout's rows (t-major, T x E): the conv1 weight gradient may then visit them env-major."""
        return FrameRingObs(self.frames, fidx, rollout_len)

    def gather_s2d(self, fidx: torch.Tensor) -> torch.Tensor:
        """The observations [n, 21, 21, 64] the frame rows ``fidx`` [n, 4] describe (tests)."""
        fr = self.frames.view(-1, 441, 4, 4)[fidx.long()]            # [n, f, pos, dy, dx]
        return fr.permute(0, 2, 3, 4, 1).reshape(-1, 21, 21, 64).contiguous()


class FrameRingObs:
    """A batch of observations as frame rows ``fidx`` [n, 4] into a ``FrameRing``'s store: what
    ``DeviceNatureCNN`` takes in place of an s2d uint8 tensor (slicing gives sub-batches)."""
    __slots__ = ("frames", "fidx", "rollout_len")

    def __init__(self, frames: torch.Tensor, fidx: torch.Tensor, rollout_len: int = 0):
        self.frames, self.fidx, self.rollout_len = frames, fidx.reshape(-1, 4), int(rollout_len)

    @property
    def shape(self):
        return (self.fidx.shape[0], 4)

    def contiguous(self):
        return FrameRingObs(self.frames, self.fidx.contiguous(), self.rollout_len)

    def __getitem__(self, sl):  # a slice is no longer a whole T x E rollout block
        return FrameRingObs(self.frames, self.fidx[sl])


class DevicePong:
    """Kernel-driven batch of PongSynth envs on one device."""

    def __init__(self, num_envs: int, device, seed: int = 0, max_steps: int = 27000 // 4):
        from ..ops import hip

        self.h = hip()
        self.N = int(num_envs)
        self.seed = int(seed) & 0x7FFFFFFFFFFFFFFF
        self.max_steps = int(max_steps)
        dev = torch.device(device)
        self.state = torch.zeros(self.N * int(self.h.pong_state_size()), device=dev)
        self.rew = torch.zeros(self.N, device=dev)
        self.done = torch.zeros(self.N, device=dev)
        self.fin_ret = torch.zeros(self.N, device=dev)
        self.fin_len = torch.zeros(self.N, device=dev)
        self.ep_acc = torch.zeros(self.N, 4, device=dev)  # per env: episodes, sum ret, sum len, sum ret^2
        self._dummy_act = torch.zeros(self.N, dtype=torch.int32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)

    # The RNG step counter lives on the device (``step_t``) so that a rollout captured in
    # a hipGraph draws fresh numbers on every replay; kernels add their host ``offset``.
    @property
    def step_count(self) -> int:
        return int(self.step_t.item())

    @step_count.setter
    def step_count(self, v: int):
        self.step_t.fill_(int(v))

    def advance(self, k: int):
        self.h.counter_add(self.step_t, int(k))

    def reset(self, obs_out: torch.Tensor = None, hist_out: torch.Tensor = None, ring=None):
        """Reset every env; the first observation is rendered into ``obs_out`` ([N, 21, 21, 64]) or,
        for the fused-render path, only its frame history goes to ``hist_out`` ([N, 16]); ``ring``
        (a ``FrameRing`` and its fidx row [N, 4]): the reset frame into the ring."""
        if ring is not None:
            fr, fidx = ring
            self.h.pong_step(self.state, self._dummy_act, self.rew, self.done, self.fin_ret, self.fin_len, None,
                             self.N, self.seed, 0, self.max_steps, True, self.step_t, frames=fr.frames, fidx=fidx,
                             ring_slots=fr.R)
        elif hist_out is not None:
            self.h.pong_step(self.state, self._dummy_act, self.rew, self.done, self.fin_ret, self.fin_len, None,
                             self.N, self.seed, 0, self.max_steps, True, self.step_t, hist=hist_out)
        else:
            self.h.pong_step(self.state, self._dummy_act, self.rew, self.done, self.fin_ret, self.fin_len, None,
                             self.N, self.seed, 0, self.max_steps, True, self.step_t, obs=obs_out)
        self.advance(1)

    def ring_fill(self, ring, fidx: torch.Tensor):
        """Rebuild the frame ring's last 4 frames and the current observation's frame rows from the
        env state alone (after a checkpoint / snapshot restore): the observation produced by the
        last step is step ``step_t - 1``."""
        self.h.pong_ring_fill(self.state, ring.frames, fidx, self.N, ring.R, -1, self.step_t)

    def episode_stats(self):
        """(episodes, sum return, sum length, sum return^2) over all envs since the last reset."""
        return self.ep_acc.double().sum(0)

    def step_head(self, part, splits: int, fc_b, head_params, A: int, h_out, act_out, logp_out, value_out,
                  sample_seed: int, sample_step: int, sample_base, obs_out, rew_out=None, done_out=None,
                  offset: int = None, ring=None):
        """The policy head fused in front of one env step (pong.hip ``pong_head_step_render_kernel``):
        from the fc split-K partials ``part`` of this step's observations, write the hidden units
        (``h_out``), sample the actions (``act_out`` / ``logp_out`` / ``value_out``, bitwise what
        ``DeviceNatureCNN.act`` gives), step every env with them and render ``obs_out`` -- or, with
        ``ring`` (a ``FrameRing``), the one new frame into the ring and the frame rows to ``obs_out``
        ([N, 4] int32)."""
        rew = self.rew if rew_out is None else rew_out
        done = self.done if done_out is None else done_out
        rk = {} if ring is None else {"frames": ring.frames, "fidx": obs_out, "ring_slots": ring.R}
        self.h.pong_head_step(part, int(splits), fc_b, head_params, int(A), h_out, act_out, logp_out, value_out,
                              int(sample_seed), int(sample_step), sample_base, self.state, rew, done, self.fin_ret,
                              self.fin_len, self.ep_acc, None if ring is not None else obs_out, self.N, self.seed,
                              0 if offset is None else int(offset), self.step_t, self.max_steps, **rk)
        if offset is None:
            self.advance(1)
        return rew, done

    def step(self, act: torch.Tensor, obs_out: torch.Tensor = None, rew_out=None, done_out=None, offset: int = None,
             hist_out: torch.Tensor = None, ring=None):
        """One env step.  Without ``offset`` the device counter is advanced after the step;
        with it (graph-captured rollouts) the caller advances once per rollout.  ``hist_out``
        ([N, 16]) instead of ``obs_out``: physics only, the new frame histories written for a
        fused-render conv stack (no 57 MB observation write per step at 2,048 envs).  ``ring`` (a
        ``FrameRing``): one new frame per env into the ring, the frame rows to ``obs_out`` ([N, 4])."""
        rew = self.rew if rew_out is None else rew_out
        done = self.done if done_out is None else done_out
        if ring is not None:  # physics + ONE new frame (7 KB instead of the 28 KB stack)
            self.h.pong_step(self.state, act, rew, done, self.fin_ret, self.fin_len, self.ep_acc, self.N, self.seed,
                             0 if offset is None else int(offset), self.max_steps, False, self.step_t,
                             frames=ring.frames, fidx=obs_out, ring_slots=ring.R)
        elif hist_out is not None:  # physics (one thread per env) + the 64-byte history row
            self.h.pong_step(self.state, act, rew, done, self.fin_ret, self.fin_len, self.ep_acc, self.N, self.seed,
                             0 if offset is None else int(offset), self.max_steps, False, self.step_t, hist=hist_out)
        else:  # physics + render of the new 4-frame stack in one launch (one workgroup per env)
            self.h.pong_step(self.state, act, rew, done, self.fin_ret, self.fin_len, self.ep_acc, self.N, self.seed,
                             0 if offset is None else int(offset), self.max_steps, False, self.step_t, obs=obs_out)
        if offset is None:
            self.advance(1)
        return rew, done
