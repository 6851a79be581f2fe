"""Nature-CNN actor-critic for pixel observations (A2C / Pong configuration, BASELINE.json
config 4 -- a model family the reference does not have; SURVEY §2.6 "New: CNN encoder").

    obs uint8 [B, 21, 21, 64]  (space-to-depth(4) of the [84, 84, 4] NHWC frame stack)
    conv 8x8/4  4 -> 32, ReLU      (84 -> 20; run as a 2x2/1 conv over the 64 s2d channels)
    conv 4x4/2 32 -> 64, ReLU      (20 -> 9)
    conv 3x3/1 64 -> 64, ReLU      (9 -> 7)
    fc 3136 -> 512, ReLU           (NHWC flatten)
    policy 512 -> A, value 512 -> 1

Parameters are ONE flat fp32 vector (master copy for Adam and the RCCL all-reduce) with
conv weights stored [Cout][KH][KW][Cin] so that the implicit-GEMM reduction index
(kh, kw, c) is contiguous in both operands (conv1 in its space-to-depth order
[32][kh2][kw2][dy][dx][c] with kh = 4*kh2 + dy, kw = 4*kw2 + dx); the device path keeps a bf16 shadow copy
of the same vector for the MFMA GEMMs (written by the fused Adam).

``DeviceNatureCNN`` runs everything through the gfx950 kernels (csrc/kernels/cnn.hip);
``reference_forward`` is the fp32 (optionally bf16-emulating) PyTorch oracle the kernels
are tested against and the CPU path of the trainer.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.nn.functional as F

# RRL_HEAD_GRID_CAP: workgroup cap of the rollout head launch (4 rows per workgroup, so rows
# past 4 x cap run 2+ rows per wave)
_HEAD_GRID_CAP = max(1, int(os.environ.get("RRL_HEAD_GRID_CAP", "1024")))

FRAME_HW = 84
FRAMES = 4
HIDDEN = 512


@dataclass(frozen=True)
class ConvLayer:
    cin: int
    cout: int
    k: int
    s: int
    hin: int

    @property
    def hout(self) -> int:
        return (self.hin - self.k) // self.s + 1

    @property
    def K(self) -> int:
        return self.k * self.k * self.cin


CONVS = (ConvLayer(FRAMES, 32, 8, 4, FRAME_HW), ConvLayer(32, 64, 4, 2, 20), ConvLayer(64, 64, 3, 1, 9))
# the geometry conv1 actually runs with on the space-to-depth input
S2D = ConvLayer(64, 32, 2, 1, 21)
OBS_S2D = (21, 21, 64)


def conv1_s2d_to_khkwc(w):
    """conv1 weights [32, 2, 2, 64] (s2d order) -> [32, 8, 8, 4] ([Cout][kh][kw][c])."""
    return w.reshape(32, 2, 2, 4, 4, 4).permute(0, 1, 3, 2, 4, 5).reshape(32, 8, 8, 4)


def conv1_khkwc_to_s2d(w):
    return w.reshape(32, 2, 4, 2, 4, 4).permute(0, 1, 3, 2, 4, 5).reshape(32, 2, 2, 64)


def obs_to_nchw(obs_u8):
    """uint8 observations (s2d [B, 21, 21, 64] or NHWC [B, 84, 84, 4]) -> float NCHW / 255."""
    if tuple(obs_u8.shape[1:]) == OBS_S2D:
        obs_u8 = obs_u8.reshape(-1, 21, 21, 4, 4, 4).permute(0, 1, 3, 2, 4, 5).reshape(-1, 84, 84, 4)
    return (obs_u8.float() / 255.0).permute(0, 3, 1, 2)
FC_IN = CONVS[-1].hout ** 2 * CONVS[-1].cout  # 3136


@dataclass(frozen=True)
class CNNSpec:
    act_dim: int = 6

    def offsets(self) -> Dict[str, int]:
        o, off = {}, 0
        for i, L in enumerate(CONVS, 1):
            o[f"w{i}"] = off
            off += L.cout * L.K
            o[f"b{i}"] = off
            off += L.cout
        o["wfc"] = off
        off += HIDDEN * FC_IN
        o["bfc"] = off
        off += HIDDEN
        o["head"] = o["wpi"] = off
        off += self.act_dim * HIDDEN
        o["bpi"] = off
        off += self.act_dim
        o["wv"] = off
        off += HIDDEN
        o["bv"] = off
        off += 1
        o["P"] = off
        return o

    @property
    def P(self) -> int:
        return self.offsets()["P"]

    @property
    def head_size(self) -> int:
        return (self.act_dim + 1) * HIDDEN + self.act_dim + 1

    def init(self, seed: int = 0, device="cpu") -> torch.Tensor:
        """Orthogonal init (gain sqrt(2) trunk, 0.01 policy, 1 value), zero biases -- the
        usual A2C/Atari recipe."""
        g = torch.Generator().manual_seed(int(seed))
        o = self.offsets()
        p = torch.zeros(o["P"])

        def orth(rows, cols, gain):
            w = torch.empty(rows, cols)
            torch.nn.init.orthogonal_(w, gain=gain, generator=g)
            return w.reshape(-1)

        for i, L in enumerate(CONVS, 1):
            p[o[f"w{i}"]:o[f"b{i}"]] = orth(L.cout, L.K, 2 ** 0.5)
        p[o["wfc"]:o["bfc"]] = orth(HIDDEN, FC_IN, 2 ** 0.5)
        p[o["wpi"]:o["bpi"]] = orth(self.act_dim, HIDDEN, 0.01)
        p[o["wv"]:o["bv"]] = orth(1, HIDDEN, 1.0)
        return p.to(device)

    def views(self, params: torch.Tensor):
        o = self.offsets()
        v = {}
        for i, L in enumerate(CONVS, 1):
            w = params[o[f"w{i}"]:o[f"b{i}"]]
            v[f"w{i}"] = conv1_s2d_to_khkwc(w) if i == 1 else w.view(L.cout, L.k, L.k, L.cin)
            v[f"b{i}"] = params[o[f"b{i}"]:o[f"b{i}"] + L.cout]
        v["wfc"] = params[o["wfc"]:o["bfc"]].view(HIDDEN, FC_IN)
        v["bfc"] = params[o["bfc"]:o["bfc"] + HIDDEN]
        v["wpi"] = params[o["wpi"]:o["bpi"]].view(self.act_dim, HIDDEN)
        v["bpi"] = params[o["bpi"]:o["bpi"] + self.act_dim]
        v["wv"] = params[o["wv"]:o["bv"]]
        v["bv"] = params[o["bv"]:o["bv"] + 1]
        v["head"] = params[o["head"]:o["P"]]
        return v


def _bf(x, emulate: bool):
    return x.to(torch.bfloat16).float() if emulate else x


def reference_forward(spec: CNNSpec, params: torch.Tensor, obs_u8: torch.Tensor, emulate_bf16: bool = False):
    """fp32 oracle.  ``emulate_bf16`` rounds weights, the scaled input and every stored
    activation to bf16 exactly where the device path does.  Returns (logits, value, acts)."""
    v = spec.views(params)
    x = _bf(obs_to_nchw(obs_u8), emulate_bf16)
    acts = []
    for i, L in enumerate(CONVS, 1):
        w = _bf(v[f"w{i}"], emulate_bf16).permute(0, 3, 1, 2)
        x = _bf(F.relu(F.conv2d(x, w, v[f"b{i}"], stride=L.s)), emulate_bf16)
        acts.append(x)
    flat = x.permute(0, 2, 3, 1).reshape(x.shape[0], FC_IN)
    h = _bf(F.relu(flat @ _bf(v["wfc"], emulate_bf16).t() + v["bfc"]), emulate_bf16)
    logits = h @ v["wpi"].t() + v["bpi"]
    value = h @ v["wv"] + v["bv"]
    return logits, value, acts + [h]


def a2c_loss(logits, value, act, adv, ret, vf_coef: float, ent_coef: float):
    logp_all = torch.log_softmax(logits, -1)
    logp = logp_all.gather(1, act.long()[:, None])[:, 0]
    ent = -(logp_all.exp() * logp_all).sum(-1)
    pg = -(adv * logp).mean()
    vf = ((value - ret) ** 2).mean()
    return pg + vf_coef * vf - ent_coef * ent.mean(), pg, vf, ent.mean()


class DeviceNatureCNN:
    """Kernel-backed model: forward (rollout + stored activations), A2C backward, Adam."""

    def __init__(self, spec: CNNSpec, device, max_batch: int, seed: int = 0, params: Optional[torch.Tensor] = None):
        from ..ops import hip, use_hip

        self.spec = spec
        self.device = torch.device(device)
        self.A = spec.act_dim
        self.max_batch = int(max_batch)
        self.params = (spec.init(seed) if params is None else params.detach().float().cpu()).to(self.device)
        if not use_hip(self.params):
            raise RuntimeError("DeviceNatureCNN needs a GPU tensor (CPU runs use reference_forward)")
        self.h = hip()
        # one fused launch for the conv stack's forward (RRL_CNN_FUSED=0: the per-layer kernels)
        import os

        self.fused_convs = os.environ.get("RRL_CNN_FUSED", "1") != "0"
        # variant of the fused forward (cnn_fused.hip, for A/B runs): 0 = the default kernel
        # (RRL_CONV_FWD, default the 16-wave one), 128 = the 8-wave kernel, 16 / 32 / 48 = its LDS layouts (a1 as phase
        # images, conv3 over a 7 x 9 grid, both); 64 = the 16-wave kernel, 80 / 96 / 112 = its layouts
        self.fwd_layout = int(os.environ.get("RRL_CNN_FWD_LAYOUT", "0"))
        assert self.fwd_layout in (0, 16, 32, 48, 64, 65, 68, 72, 73, 80, 96, 112, 128), "RRL_CNN_FWD_LAYOUT"
        # conv2 backward variant (A/B runs): 0 = dgrad over 7 tiles per class, 2 = a 10 x 12 grid
        self.bwd2_variant = int(os.environ.get("RRL_CNN_BWD2_VARIANT", "0"))
        assert self.bwd2_variant in (0, 2, 3, 4, 5, 6, 7, 8), \
            "RRL_CNN_BWD2_VARIANT: 0, 2, 3 (16 waves), 4-7 (wave priority), 8 (16-byte da1 stores)"
        self.bwd3_variant = int(os.environ.get("RRL_CNN_BWD3_VARIANT", "0"))
        # resident conv3-backward workgroups per CU (RRL_CNN_BWD3_WGS, A/B runs): its 74,880 B of
        # LDS and 128 VGPRs leave room for a second one
        self.bwd3_wgs = max(1, min(2, int(os.environ.get("RRL_CNN_BWD3_WGS", "1"))))
        assert self.bwd3_variant in (0, 1, 2, 3, 4, 5, 6), \
            "RRL_CNN_BWD3_VARIANT: 0 (s_setprio clusters), 1 (16 waves), 2 (no s_setprio), 3 (static), 4 / 5 (one cluster)"
        # conv2 backward + conv1 weight gradient in C row chunks, each chunk's da1 read back by
        # conv1_wgrad8 right after conv2_bwd wrote it (RRL_CNN_BWD21_CHUNKS, for A/B runs: a half
        # batch's da1 fits the 256 MB Infinity Cache, the whole one does not at 10,240 frames)
        self.bwd21_chunks = max(1, int(os.environ.get("RRL_CNN_BWD21_CHUNKS", "1")))
        # fc layer on the DMA-staged NT GEMM (fc.hip): forward as split-K partials reduced by
        # the head kernel (bias + ReLU + bf16 + logits / value / sample in one launch), data
        # gradient against a transposed bf16 shadow of Wfc (RRL_FC_NT=0: the gemm_bf16.h path)
        self.fc_nt = os.environ.get("RRL_FC_NT", "1") != "0"
        # fc bias gradient inside the weight-gradient GEMM (a ones column in its padded tile)
        self.fc_tn_bias = os.environ.get("RRL_FC_TN_BIAS", "1") != "0"
        self.o = spec.offsets()
        self.P = self.o["P"]
        dev = self.device
        self.shadow = torch.empty(self.P, dtype=torch.bfloat16, device=dev)
        self.wfc_t = torch.empty(FC_IN * HIDDEN, dtype=torch.bfloat16, device=dev)  # [3136][512]
        # split-K partials of the fc forward, sized once for every batch up to max_batch: a
        # captured update graph holds this storage, so it must never be reallocated
        self.FC_SPLIT_CAP = int(os.environ.get("RRL_FC_SPLITS", str(self.FC_SPLIT_CAP)))
        fc_rows = (max(self.fc_splits(n, big) * n for n in range(1, self.max_batch + 1) for big in (False, True))
                   if self.fc_nt else 0)
        self._fc_part = torch.empty(fc_rows * HIDDEN, device=dev) if self.fc_nt else None
        self.refresh_shadow()
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.grad = torch.zeros_like(self.params)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)  # Adam step (device: graph replays)
        B = self.max_batch
        bf = torch.bfloat16
        L1, L2, L3 = CONVS
        self.a1 = torch.empty(B * L1.hout ** 2 * L1.cout, dtype=bf, device=dev)
        self.a2 = torch.empty(B * L2.hout ** 2 * L2.cout, dtype=bf, device=dev)
        self.a3 = torch.empty(B * FC_IN, dtype=bf, device=dev)
        self.hid = torch.empty(B * HIDDEN, dtype=bf, device=dev)
        # backward buffers
        self.dh = torch.empty(B * HIDDEN, dtype=bf, device=dev)
        self.da3 = torch.empty(B * FC_IN, dtype=bf, device=dev)
        self.da2 = torch.empty(B * L2.hout ** 2 * L2.cout, dtype=bf, device=dev)
        self.da1 = torch.empty(B * L1.hout ** 2 * L1.cout, dtype=bf, device=dev)
        self.dhead = torch.empty(B * (self.A + 1), dtype=torch.float32, device=dev)
        self.head_grid = max(1, min(1024, (B + 3) // 4))
        # backward head: rows per wave (RRL_HEAD_BWD_ROWS, for A/B runs; grid = B / (4 x rows))
        self.head_bwd_rows = max(1, int(os.environ.get("RRL_HEAD_BWD_ROWS", "4")))
        self.stats = torch.empty(max(self.head_grid, (B + 3) // 4) * 4, device=dev)
        self.head_blocks = max(1, min(256, (B + 31) // 32))
        self.head_part = torch.empty(self.head_blocks * spec.head_size, device=dev)
        # split-K plan for the weight gradients (enough workgroups to fill 256 CUs)
        self._wplan = {}
        need = self.head_blocks * spec.head_size
        for name, cout, K, M in self._wgrad_layers(B):
            tiles = -(-K // 128) * -(-cout // (64 if cout >= 64 else 32))
            s = int(self.h.gemm_splits(M, max(1, min(512 // max(tiles, 1), -(-M // 64)))))
            self._wplan[name] = s
            need = max(need, s * cout * K)
        self.cus = int(self.h.device_cus())
        need = max(need, min(B, self.cus * self.bwd3_wgs) * CONVS[2].cout * CONVS[2].K)  # fused conv3 backward partials
        if self.fc_nt:
            need = max(need, self.FC_WGRAD_SPLITS * HIDDEN * FC_IN)
            self._ones8 = torch.ones(8, dtype=torch.bfloat16, device=dev)
            self._fc_bias_part = torch.empty(self.FC_WGRAD_SPLITS * HIDDEN, device=dev)
        self.part = torch.empty(need, device=dev)
        self.bias_splits = 512
        self.bias_part = torch.empty(max(self.bias_splits * HIDDEN, self.cus * 512), device=dev)
        if self.fused_convs:
            # per-layer partial slabs of the fused conv backward kernels, summed together in ONE
            # launch at the end of the backward (sum_splits_multi)
            nb = min(B, self.cus)
            C = self.bwd21_chunks
            L1_, L2_, L3_ = CONVS
            nb3 = min(B, self.cus * self.bwd3_wgs)
            self.cpart = {"c3": torch.empty(nb3 * L3_.cout * L3_.K, device=dev),
                          "c2": torch.empty(C * nb * L2_.cout * L2_.K, device=dev),
                          "c1": torch.empty(C * 2 * nb * S2D.cout * S2D.K, device=dev)}  # 2 slabs per workgroup
            # bias partials: 64 per workgroup written, 512 per workgroup checked by the binding
            self.cbias = {"c3": torch.empty(nb3 * 8 * L3_.cout, device=dev),
                          "c2": torch.empty((C + 1) * nb * 8 * L2_.cout, device=dev),
                          "c1": torch.empty(C * 2 * nb * S2D.cout, device=dev)}
        self.sq_work = torch.empty(1024, device=dev)
        # side stream for the head / fc weight gradients (backward, one rank; RRL_CNN_SIDE=0: off)
        self.side_stream = torch.cuda.Stream(device=dev) if os.environ.get("RRL_CNN_SIDE", "1") != "0" else None
        # what the side stream takes (RRL_CNN_SIDE_MODE): "early" = head + fc weight gradients
        # forked before the fc data gradient (the two fc GEMMs share the chip); "late" = the
        # same work forked after it (beside conv3_bwd); "sums" = both fc GEMMs back to back on
        # the main stream and only the memory-light head gradient + split sums forked beside
        # conv3_bwd; "early_main" (default) = "early" with the side work captured AFTER the fc data
        # gradient: same graph edges, but the replay now dispatches the main branch's kernel
        # first (fork gap on the main stream 14 -> 6 us, join 10 -> 6 us; Pong +2.3 % at 2,048
        # envs, +-0 at 8,192: profiles/r5_pong_side_early_main_ab.txt)
        # "c3" = the side work forked after the conv3 backward (beside conv2 / conv1)
        self.side_mode = os.environ.get("RRL_CNN_SIDE_MODE", "early_main")
        if os.environ.get("RRL_CNN_SIDE_LATE", "0") == "1":
            self.side_mode = "late"
        assert self.side_mode in ("early", "early_main", "late", "sums", "c3"), self.side_mode
        self._ev_fork = torch.cuda.Event()
        self._ev_join = torch.cuda.Event()
        self._ev_c3, self._ev_c3_done = torch.cuda.Event(), torch.cuda.Event()
        self._ev_c2, self._ev_c2_done = torch.cuda.Event(), torch.cuda.Event()
        # RRL_CNN_SIDE_CONV_SUMS=1 (off): see backward(); ABBA -0.0 / -0.4 % at 2,048 / 8,192 envs
        self.side_conv_sums = os.environ.get("RRL_CNN_SIDE_CONV_SUMS", "0") == "1"
        # RRL_CNN_SIDE_FC_FIRST=1: the side stream runs the fc weight GEMM before the head gradient
        # (the GEMM then overlaps the fc data gradient more: -2.3 % at 2,048 / 8,192 envs)
        self.side_fc_first = os.environ.get("RRL_CNN_SIDE_FC_FIRST", "0") == "1"
        self._ev_t_fork = torch.cuda.Event()
        self._ev_t_join = torch.cuda.Event()
        self._wfc_t_stale = self._wfc_t_pending = False
        # RRL_CNN_DEFER_TRANSPOSE=1: the transposed-Wfc refresh after Adam moves to the side stream
        # beside the next rollout -- +0.3 % at 2,048 envs, -0.5 % at 8,192 in an ABBA run
        # (profiles/r4_defer_transpose_ab.txt): off by default
        self.defer_transpose = os.environ.get("RRL_CNN_DEFER_TRANSPOSE", "0") == "1"
        self.norm_sq = torch.empty(1, device=dev)

    @staticmethod
    def _wgrad_layers(B):
        L1, L2, L3 = CONVS
        return [("fc", HIDDEN, FC_IN, B), ("c3", L3.cout, L3.K, B * L3.hout ** 2),
                ("c2", L2.cout, L2.K, B * L2.hout ** 2), ("c1", L1.cout, L1.K, B * L1.hout ** 2)]

    # ------------------------------------------------------------------ forward
    def _rows(self, buf, row0, rows, per_row):
        return buf[row0 * per_row:(row0 + rows) * per_row]

    def refresh_shadow(self):
        """bf16 copies of the fp32 master weights (after a load / broadcast; Adam writes the
        flat shadow itself) and the transposed fc shadow for the data gradient."""
        if getattr(self, "_wfc_t_pending", False):
            self._wfc_t_ready()  # a side-stream refresh in flight finishes first
        self.h.to_bf16(self.params, self.shadow)
        self._transpose_fc()
        self._wfc_t_stale = False

    def _transpose_fc(self):
        o = self.o
        self.h.transpose_bf16(self.shadow[o["wfc"]:o["bfc"]], self.wfc_t, HIDDEN, FC_IN)

    # fc weight gradient (fc_tn_part): 100 output tiles x 5 row splits = 500 workgroups, two
    # per CU (tools/fc_kbench.py)
    FC_WGRAD_SPLITS = 5

    # cap of the fc forward's split-K count (RRL_FC_SPLITS, for A/B runs)
    FC_SPLIT_CAP = 8

    def fc_splits(self, n: int, big=None) -> int:
        """split-K count of the fc forward: enough items for 256 CUs, at most 8 -- of the
        persistent 256 x 128 tiles (fc.hip ``fcp_nt_kernel``: >= 4,096 rows, or RRL_FC_BIG=1)
        or of the 128 x 128 one-tile-per-workgroup kernel."""
        if big is None:  # the same choice as fc.hip's rrl_fc_nt_part
            e = os.environ.get("RRL_FC_BIG", "")
            big = (e != "0") if e else n >= 4096
        tiles = -(-n // (256 if big else 128)) * (HIDDEN // 128)
        return max(1, min(self.FC_SPLIT_CAP, -(-256 // tiles)))

    @staticmethod
    def _head_grid(n: int) -> int:
        """Workgroups of the rollout head launch: one row per wave, 4 waves each (2 or 4 rows per
        wave measured 1.5 / 5 % slower per update: profiles/r4_head_rows_ab.txt)."""
        return max(1, min(_HEAD_GRID_CAP, (n + 3) // 4))

    def _fc_head(self, a3, hid, n, **head):
        """fc GEMM as split-K partials, then ONE head launch: bias + ReLU + bf16 hid (stored for
        the backward) + logits / value / sampling."""
        o = self.o
        s = self.fc_splits(n)
        assert s * n * HIDDEN <= self._fc_part.numel(), "fc split-K partials exceed the preallocated buffer"
        used = int(self.h.fc_nt_part(a3, self.shadow[o["wfc"]:o["bfc"]], self._fc_part, n, HIDDEN, FC_IN, s))
        self.h.a2c_head(0, hid, self.params[o["head"]:], n, self.A, head.get("act"), head.get("logp"),
                        head.get("value"), head.get("logits"), int(head.get("seed", 0)), int(head.get("step", 0)),
                        int(head.get("row_offset", 0)), None, None, None, 0.0, 0.0, 0.0, None, None, None,
                        self._head_grid(n), head.get("step_base"), part=self._fc_part, splits=used,
                        fc_b=self.params[o["bfc"]:o["bfc"] + HIDDEN])

    @staticmethod
    def is_hist(obs) -> bool:
        """PongSynth frame histories [n, 16] float32 (4 frames x (bx, by, pa, po)) instead of s2d
        frames: the fused-render path, where the conv kernels draw the observation themselves."""
        return torch.is_tensor(obs) and obs.dtype == torch.float32 and obs.dim() == 2 and obs.shape[1] == 16

    @staticmethod
    def is_ring(obs) -> bool:
        """Frame-ring observations (``envs.pong.FrameRingObs``): frame rows into a frame store, read
        and interleaved by the conv kernels themselves (csrc/kernels/pong_render.h)."""
        return hasattr(obs, "fidx") and hasattr(obs, "frames")

    @classmethod
    def _c1_src(cls, x) -> dict:
        """The conv1 weight gradient's frame source keywords for observations ``x``.  Frame-ring
        rows of a whole T-step rollout are visited env-major from 4,096 envs (the T observations of
        one env share frames, which then come from the CU's L2): at 8,192 envs that measured
        493.7 -> 486.9 us per launch, at 2,048 -- whose ring, 130 MB, stays in the Infinity Cache
        anyway -- 126.5 -> 129.9 us (profiles/r6_pong_ring_v4_ab.txt).  RRL_CNN_WGRAD1_ENV_MAJOR =
        1 / 0 forces it on / off."""
        if cls.is_ring(x):
            kw = {"frames": x.frames, "fidx": x.fidx}
            T = getattr(x, "rollout_len", 0)
            em = os.environ.get("RRL_CNN_WGRAD1_ENV_MAJOR", "")
            if T > 1 and x.fidx.shape[0] % T == 0 and (em == "1" or (em == "" and x.fidx.shape[0] // T >= 4096)):
                kw["env_major_T"] = T
            return kw
        if cls.is_hist(x):
            return {"hist": x}
        return {}

    def forward(self, obs_u8: torch.Tensor, row0: int = 0, fc: bool = True, store_acts: bool = True):
        """Conv stack + fc on obs [n, 84, 84, 4]; activations land in rows row0.. of the
        stored buffers.  Returns the hidden [n * 512] view (with fc=False only the conv
        stack runs and the view is not written yet).  store_acts=False: a1 / a2 are not
        written (a forward no backward reads, e.g. the bootstrap value; fused path only).
        ``obs_u8`` may be PongSynth frame histories [n, 16] (``is_hist``): the 16-wave conv stack
        then renders the frames in LDS and no observation tensor exists."""
        n = obs_u8.shape[0]
        assert row0 + n <= self.max_batch, "batch exceeds the model's activation buffers"
        h, o, sh, p = self.h, self.o, self.shadow, self.params
        L1, L2, L3 = CONVS
        a1 = self._rows(self.a1, row0, n, L1.hout ** 2 * L1.cout)
        a2 = self._rows(self.a2, row0, n, L2.hout ** 2 * L2.cout)
        a3 = self._rows(self.a3, row0, n, FC_IN)
        hid = self._rows(self.hid, row0, n, HIDDEN)
        x = obs_u8.contiguous()
        if self.is_ring(x):
            assert self.fused_convs and self.fwd_layout in (0, 64), "frame ring: the 16-wave conv stack only"
            h.conv_stack_fwd(None, *(t for i in (1, 2, 3) for t in (sh[o[f"w{i}"]:o[f"b{i}"]],
                                                                        p[o[f"b{i}"]:o[f"b{i}"] + CONVS[i - 1].cout])),
                             a1, a2, a3, n, store12=store_acts, frames=x.frames, fidx=x.fidx)
        elif self.is_hist(x):
            assert self.fused_convs and self.fwd_layout in (0, 64), "fused render: the 16-wave conv stack only"
            h.conv_stack_fwd(None, *(t for i in (1, 2, 3) for t in (sh[o[f"w{i}"]:o[f"b{i}"]],
                                                                        p[o[f"b{i}"]:o[f"b{i}"] + CONVS[i - 1].cout])),
                             a1, a2, a3, n, store12=store_acts, hist=x)
        elif self.fused_convs:
            assert tuple(x.shape[1:]) == OBS_S2D, "device CNN takes space-to-depth observations [n, 21, 21, 64]"
            # conv1 -> conv2 -> conv3 in one launch, activations LDS-resident (cnn_fused.hip)
            h.conv_stack_fwd(x, *(t for i in (1, 2, 3) for t in (sh[o[f"w{i}"]:o[f"b{i}"]],
                                                                     p[o[f"b{i}"]:o[f"b{i}"] + CONVS[i - 1].cout])),
                             a1, a2, a3, n, probe=self.fwd_layout, store12=store_acts)
        else:
            for i, (L, y) in enumerate(zip((S2D,) + CONVS[1:], (a1, a2, a3)), 1):
                h.conv_fwd(x, sh[o[f"w{i}"]:o[f"b{i}"]], p[o[f"b{i}"]:o[f"b{i}"] + L.cout], y, n, L.hin, L.hin,
                           L.cin, L.k, L.k, L.s, L.cout, True)
                x = y
        if fc:
            h.conv_fwd(a3, sh[o["wfc"]:o["bfc"]], p[o["bfc"]:o["bfc"] + HIDDEN], hid, n, 1, 1, FC_IN, 1, 1, 1,
                       HIDDEN, True, self.part)  # split-K when the batch is too small to fill the chip
        return hid

    def forward_fc_partials(self, obs_u8, row0: int):
        """Conv stack + the fc GEMM's split-K partials for rows row0.. (no head): the fused Pong
        rollout step (``DevicePong.step_head``) forms the hidden units and samples from them.
        Returns (partials, splits used, hidden-unit view [n * 512] the head writes)."""
        assert self.fc_nt, "the fused head needs the split-K fc (RRL_FC_NT=1)"
        n = obs_u8.shape[0]
        hid = self.forward(obs_u8, row0, fc=False)
        s = self.fc_splits(n)
        assert s * n * HIDDEN <= self._fc_part.numel(), "fc split-K partials exceed the preallocated buffer"
        used = int(self.h.fc_nt_part(self._rows(self.a3, row0, n, FC_IN), self.shadow[self.o["wfc"]:self.o["bfc"]],
                                     self._fc_part, n, HIDDEN, FC_IN, s))
        return self._fc_part, used, hid

    def head_params(self):
        """(fc bias [512], head parameters: A policy rows | A biases | value row | value bias)."""
        o = self.o
        return self.params[o["bfc"]:o["bfc"] + HIDDEN], self.params[o["head"]:]

    def _forward_head(self, obs_u8, row0, store_acts=True, **head):
        n = obs_u8.shape[0]
        if self.fc_nt:
            hid = self.forward(obs_u8, row0, fc=False, store_acts=store_acts)
            self._fc_head(self._rows(self.a3, row0, n, FC_IN), hid, n, **head)
            return
        hid = self.forward(obs_u8, row0)
        self.h.a2c_head(0, hid, self.params[self.o["head"]:], n, self.A, head.get("act"), head.get("logp"),
                        head.get("value"), head.get("logits"), int(head.get("seed", 0)), int(head.get("step", 0)),
                        int(head.get("row_offset", 0)), None, None, None, 0.0, 0.0, 0.0, None, None, None,
                        self._head_grid(n), head.get("step_base"))

    def act(self, obs_u8, row0, act_out, logp_out, value_out, seed: int, step: int, row_offset: int = 0,
            step_base=None):
        """Sample actions; the Philox step is ``step`` (+ the device counter ``step_base``)."""
        self._forward_head(obs_u8, row0, act=act_out, logp=logp_out, value=value_out, seed=seed, step=step,
                           row_offset=row_offset, step_base=step_base)

    def value(self, obs_u8, row0, value_out):
        """V(obs) into value_out (the rollout's bootstrap): no a1 / a2 stores, no backward reads them."""
        self._forward_head(obs_u8, row0, store_acts=False, value=value_out)

    def logits(self, obs_u8):
        n = obs_u8.shape[0]
        lg = torch.empty(n, self.A, device=self.device)
        val = torch.empty(n, device=self.device)
        self._forward_head(obs_u8, 0, value=val, logits=lg)
        return lg, val

    # ------------------------------------------------------------------ backward
    def backward(self, obs_u8: torch.Tensor, act: torch.Tensor, adv: torch.Tensor, ret: torch.Tensor,
                 vf_coef: float, ent_coef: float, comm=None) -> torch.Tensor:
        """A2C gradients into ``self.grad`` from the activations stored by ``forward`` for
        rows 0..B-1.  Returns the per-block loss stats [grid, 4] (pg, vf, ent, count).

        With ``comm`` (world > 1) the data-parallel all-reduce is bucketed and overlapped
        with the backward: the fc + head bucket (96 % of the 1.7 M gradient floats) is
        all-reduced asynchronously on RCCL's stream as soon as it is final, while the conv
        gradients are still being computed; the conv bucket follows at the end."""
        self._reduced = False
        pending = None
        h, o, sh, g = self.h, self.o, self.shadow, self.grad
        B = obs_u8.shape[0]
        L1, L2, L3 = CONVS
        a1 = self.a1[:B * L1.hout ** 2 * L1.cout]
        a2 = self.a2[:B * L2.hout ** 2 * L2.cout]
        a3 = self.a3[:B * FC_IN]
        hid = self.hid[:B * HIDDEN]
        dh = self.dh[:B * HIDDEN]
        dhead = self.dhead[:B * (self.A + 1)]
        r = self.head_bwd_rows  # ~4 rows per wave by default: the head weights load once per wave
        grid = max(1, min(self.stats.numel() // 4, (B + 4 * r - 1) // (4 * r)))
        stats = self.stats[:grid * 4]
        h.a2c_head(1, hid, self.params[o["head"]:], B, self.A, None, None, None, None, 0, 0, 0, act, adv, ret,
                   1.0 / B, float(vf_coef), float(ent_coef), dh, dhead, stats, grid)
        nb = max(1, min(self.head_blocks, B))
        hp = self.head_part[:nb * self.spec.head_size]
        # The head / fc weight gradients depend only on (dh, dhead, hid, a3), not on the conv
        # chain below: on one rank they run on a side stream, concurrently with the fc data
        # gradient and the conv backward (their buffers -- head_part, part, bias_part -- are
        # not touched by the fused conv path, which has its own slabs).  The DP path keeps one
        # stream: its fc bucket all-reduce is issued as soon as these gradients are final.
        side = (self.side_stream if (self.side_stream is not None and self.fused_convs and self.fc_nt
                                     and B % 64 == 0 and (comm is None or not comm.multi)) else None)

        fc_tn_used = []

        def fc_tn():  # weight AND bias gradient of fc in one GEMM: the padded last column tile
            # of a3 reads a column of ones, so its first pad column holds the column sums of dh
            fc_tn_used.append(int(h.fc_tn_part(dh, a3, self.part, B, HIDDEN, FC_IN, self.FC_WGRAD_SPLITS,
                                               ones=self._ones8, bias_part=self._fc_bias_part)))

        def head_grads():
            h.head_wgrad(hid, dhead, B, self.A, hp, nb)
            h.sum_splits(hp, nb, self.spec.head_size, g[o["head"]:o["P"]])

        def weight_grads():  # head + fc weight / bias gradients
            if not self.side_fc_first:
                head_grads()
            fc_grads()
            if self.side_fc_first:
                head_grads()

        def fc_grads():
            if self.fc_nt and B % 64 == 0 and self.fc_tn_bias:
                if not fc_tn_used:  # side mode "sums" ran the GEMM on the main stream already
                    fc_tn()
                used = fc_tn_used[0]
                h.sum_splits_multi([(self.part, used, HIDDEN * FC_IN, g[o["wfc"]:o["bfc"]]),
                                    (self._fc_bias_part, used, HIDDEN, g[o["bfc"]:o["bfc"] + HIDDEN])])
            elif self.fc_nt and B % 64 == 0:
                used = int(h.fc_tn_part(dh, a3, self.part, B, HIDDEN, FC_IN, self.FC_WGRAD_SPLITS))
                h.sum_splits(self.part, used, HIDDEN * FC_IN, g[o["wfc"]:o["bfc"]])
                self._bias(dh, B, HIDDEN, o["bfc"])
            else:
                self._wgrad("fc", dh, a3, B, 1, FC_IN, 1, 1, HIDDEN, o["wfc"])
                self._bias(dh, B, HIDDEN, o["bfc"])

        def fork_weight_grads(recorded=False):
            if side is None:
                weight_grads()
                return
            if not recorded:
                self._ev_fork.record()
            side.wait_event(self._ev_fork)
            with torch.cuda.stream(side):
                weight_grads()
                self._ev_join.record(side)
            side_last[0] = self._ev_join  # (mode "c3" forks after the conv slab sums' forks)

        # side mode "late": fork after the fc data gradient instead, so the side work runs
        # beside the latency-bound conv3 backward rather than the 2,000-workgroup fc GEMM -- +0.5 %
        # on one box, -3 to -3.4 % at 2,048 / 8,192 envs alternated on another
        # (profiles/r4_side_late_and_configs.txt, r4_side_late_ab.txt).  Mode "sums": the fc
        # weight GEMM runs right after the data GEMM on the main stream (in "early" the two
        # overlap and stretch each other: 48 + 42 us alone, ~126 us together in the trace)
        # RRL_CNN_SIDE_CONV_SUMS=1: each conv layer's slab sum forks onto the side stream as soon
        # as its backward kernel is done (conv3's beside conv2's backward, conv2's beside conv1's),
        # leaving only conv1's sum on the main stream's tail: the tail sum 23 -> 6 us, but every
        # cross-stream edge of the replayed graph costs the main stream ~9 us (kernel trace:
        # conv3 -> conv2 and conv2 -> conv1 gaps of 9-10 us), so no gain (profiles/r4_side_conv_sums_ab.txt)
        side_sums = side is not None and self.fused_convs and self.side_conv_sums

        side_last = [self._ev_join]  # the side stream's last join event (one event per record)

        def fork_sums(segs, ev, ev_done):
            ev.record()
            side.wait_event(ev)
            with torch.cuda.stream(side):
                h.sum_splits_multi(segs)
                ev_done.record(side)
            side_last[0] = ev_done

        mode = self.side_mode if side is not None else "early"
        sums_mode = mode == "sums" and self.fc_nt and B % 64 == 0 and self.fc_tn_bias
        if mode == "early" or (mode == "sums" and not sums_mode):
            fork_weight_grads()
        elif mode == "early_main":
            self._ev_fork.record()
        da3 = self.da3[:B * FC_IN]
        if self.fc_nt:
            self._wfc_t_ready()
            h.fc_nt_mask(dh, self.wfc_t, a3, da3, B, FC_IN, HIDDEN)
        else:
            h.gemm_dgrad(dh, sh[o["wfc"]:o["bfc"]], a3, da3, B, HIDDEN, FC_IN)
        if sums_mode:
            fc_tn()
        if mode == "late" or sums_mode:
            fork_weight_grads()
        elif mode == "early_main":
            fork_weight_grads(recorded=True)
        if comm is not None and comm.multi:
            import torch.distributed as dist

            pending = dist.all_reduce(g[o["wfc"]:o["P"]], group=comm.group, async_op=True)
        # conv3
        da2 = self.da2[:B * L2.hout ** 2 * L2.cout]
        if self.fused_convs:
            # dgrad + wgrad + bias in one pass over (da3, a2) per image (cnn_fused.hip); the
            # slab sums of all three conv layers run in one launch at the end
            nblk = min(B, self.cus * self.bwd3_wgs)
            h.conv3_bwd(da3, sh[o["w3"]:o["b3"]], a2, da2, self.cpart["c3"], self.cbias["c3"], B, nblk,
                        variant=self.bwd3_variant)
            sums = [(self.cpart["c3"], nblk, L3.cout * L3.K, g[o["w3"]:o["b3"]]),
                    (self.cbias["c3"], nblk, L3.cout, g[o["b3"]:o["b3"] + L3.cout])]
            if side_sums:  # conv3's slabs are final: summed on the side stream beside conv2 / conv1
                fork_sums(sums, self._ev_c3, self._ev_c3_done)
                sums = []
        else:
            self._wgrad("c3", da3, a2, B, L3.hin, L3.cin, L3.k, L3.s, L3.cout, o["w3"])
            self._bias(da3, B * L3.hout ** 2, L3.cout, o["b3"])
            self._dgrad(da3, sh[o["w3"]:o["b3"]], a2, da2, B, L3)
        if mode == "c3":
            self._ev_fork.record()
        # conv2
        da1 = self.da1[:B * L1.hout ** 2 * L1.cout]
        c1_slabs = None
        if self.fused_convs and self.bwd21_chunks > 1 and not side_sums:
            # conv2 backward + conv1 weight gradient chunk by chunk; each chunk's partial slabs
            # follow the previous chunk's, so the one slab sum at the end covers them all
            C = self.bwd21_chunks
            n2 = n1 = 0
            S2, S1, P2, P1 = L2.cout * L2.K, S2D.cout * S2D.K, L2.hout ** 2 * L2.cout, L1.hout ** 2 * L1.cout
            x8 = obs_u8.contiguous()
            raw = not (self.is_hist(x8) or self.is_ring(x8))
            for k in range(C):
                b0, b1 = B * k // C, B * (k + 1) // C
                nk = b1 - b0
                if nk < 1:
                    continue
                nblk = min(nk, self.cus)
                h.conv2_bwd(da2[b0 * P2:b1 * P2], sh[o["w2"]:o["b2"]], a1[b0 * P1:b1 * P1], da1[b0 * P1:b1 * P1],
                            self.cpart["c2"][n2 * S2:], self.cbias["c2"][n2 * L2.cout:], nk, nblk,
                            staged=self.bwd2_variant)
                n2 += nblk
                n1 += int(h.conv1_wgrad8(x8[b0:b1] if raw else None, da1[b0 * P1:b1 * P1], self.cpart["c1"][n1 * S1:],
                                         self.cbias["c1"][n1 * S2D.cout:], nk, nblk, **self._c1_src(x8[b0:b1])))
            sums += [(self.cpart["c2"], n2, S2, g[o["w2"]:o["b2"]]),
                     (self.cbias["c2"], n2, L2.cout, g[o["b2"]:o["b2"] + L2.cout])]
            c1_slabs = n1
        elif self.fused_convs:
            nblk = min(B, self.cus)
            h.conv2_bwd(da2, sh[o["w2"]:o["b2"]], a1, da1, self.cpart["c2"], self.cbias["c2"], B, nblk,
                        staged=self.bwd2_variant)
            sums += [(self.cpart["c2"], nblk, L2.cout * L2.K, g[o["w2"]:o["b2"]]),
                     (self.cbias["c2"], nblk, L2.cout, g[o["b2"]:o["b2"] + L2.cout])]
            if side_sums:
                fork_sums(sums, self._ev_c2, self._ev_c2_done)
                sums = []
        else:
            self._wgrad("c2", da2, a1, B, L2.hin, L2.cin, L2.k, L2.s, L2.cout, o["w2"])
            self._bias(da2, B * L2.hout ** 2, L2.cout, o["b2"])
            self._dgrad(da2, sh[o["w2"]:o["b2"]], a1, da1, B, L2)
        if mode == "c3":  # captured after conv2's kernels: the replay dispatches them first
            fork_weight_grads(recorded=True)
        # conv1 (input = frames, no data gradient)
        # (its bias gradient comes out of the same pass over da1)
        if self.fused_convs:
            x8 = obs_u8.contiguous()
            raw = not (self.is_hist(x8) or self.is_ring(x8))
            ns = c1_slabs if c1_slabs is not None else int(
                h.conv1_wgrad8(x8 if raw else None, da1, self.cpart["c1"], self.cbias["c1"], B, min(B, self.cus),
                               **self._c1_src(x8)))
            sums += [(self.cpart["c1"], ns, S2D.cout * S2D.K, g[o["w1"]:o["b1"]]),
                     (self.cbias["c1"], ns, S2D.cout, g[o["b1"]:o["b1"] + S2D.cout])]
            h.sum_splits_multi(sums)
        else:
            self._wgrad("c1", da1, obs_u8.contiguous(), B, S2D.hin, S2D.cin, S2D.k, S2D.s, S2D.cout, o["w1"],
                        bias_off=o["b1"])
        if side is not None:
            torch.cuda.current_stream().wait_event(side_last[0])
        if pending is not None:
            comm.all_reduce_sum_(g[:o["wfc"]])
            pending.wait()
            g.mul_(1.0 / comm.world)
            self._reduced = True
        return stats.view(grid, 4)

    def _dgrad(self, dy, w, xact, dx, B, L):
        """dX * (X > 0): implicit phase-class GEMM when the geometry has one, else an
        explicit column buffer + col2im (allocated on first use)."""
        if self.h.conv_dgrad(dy, w, xact, dx, B, L.hin, L.hin, L.cin, L.k, L.k, L.s, L.cout):
            return
        n = B * L.hout ** 2 * L.K
        if getattr(self, "_dcol", None) is None or self._dcol.numel() < n:
            self._dcol = torch.empty(self.max_batch * L.hout ** 2 * L.K, dtype=torch.bfloat16, device=self.device)
        dcol = self._dcol[:n]
        self.h.gemm_dgrad(dy, w, None, dcol, B * L.hout ** 2, L.cout, L.K)
        self.h.col2im_mask(dcol, xact, dx, B, L.hin, L.hin, L.cin, L.k, L.k, L.s)

    def _wgrad(self, name, dy, x, N, H, C, k, s, cout, off, bias_off=None):
        K = k * k * C
        bp = self.bias_part if bias_off is not None else None
        splits = int(self.h.conv_wgrad(dy, x, self.part, self._wplan[name], N, H, H, C, k, k, s, cout, bp))
        self.h.sum_splits(self.part, splits, cout * K, self.grad[off:off + cout * K])
        if bias_off is not None:
            self.h.sum_splits(self.bias_part, splits, cout, self.grad[bias_off:bias_off + cout])

    def _bias(self, dy, M, C, off):
        s = self.bias_splits
        self.h.colsum(dy, M, C, self.bias_part, s)
        self.h.sum_splits(self.bias_part, s, C, self.grad[off:off + C])

    # ------------------------------------------------------------------ optimizer
    def apply(self, lr: float, max_grad_norm: float = 0.5, comm=None, betas=(0.9, 0.999), eps: float = 1e-5,
              step_bumped: bool = False):
        """(DP all-reduce) -> global-norm clip -> Adam -> bf16 shadow, all on device.
        ``step_bumped``: the caller already advanced ``step_t`` (folded into another launch)."""
        if comm is not None and comm.multi and not getattr(self, "_reduced", False):
            comm.all_reduce_sum_(self.grad)
            self.grad.mul_(1.0 / comm.world)
        self._reduced = False
        # sum-of-squares partials; the clip + Adam launch reduces them itself (one launch fewer)
        parts = int(self.h.sumsq_partial(self.grad, self.sq_work)) if max_grad_norm > 0 else 0
        if not step_bumped:
            self.h.counter_add(self.step_t, 1)
        self.h.adam_clip(self.params, self.m, self.v, self.grad, self.shadow,
                         self.sq_work if max_grad_norm > 0 else None, float(max_grad_norm), float(lr),
                         float(betas[0]), float(betas[1]), float(eps), 0, self.step_t, norm_parts=parts)
        if self.fc_nt:
            if self.side_stream is not None and self.defer_transpose:
                # the transposed Wfc shadow is first read by the next backward's fc data gradient:
                # begin_update() runs the transpose on the side stream beside the rollout
                self._wfc_t_stale = True
            else:
                self._transpose_fc()

    def begin_update(self):
        """Start of an update (before its rollout): a transposed-Wfc refresh left by the last
        apply() runs on the side stream, joined before the backward's fc data gradient."""
        if self._wfc_t_stale and self.side_stream is not None and not self._wfc_t_pending:
            self._ev_t_fork.record()
            self.side_stream.wait_event(self._ev_t_fork)
            with torch.cuda.stream(self.side_stream):
                self._transpose_fc()
                self._ev_t_join.record(self.side_stream)
            self._wfc_t_stale, self._wfc_t_pending = False, True

    def _wfc_t_ready(self):
        """Order the transposed Wfc shadow before its first reader."""
        if self._wfc_t_pending:
            torch.cuda.current_stream().wait_event(self._ev_t_join)
            self._wfc_t_pending = False
        elif self._wfc_t_stale:
            self._transpose_fc()
            self._wfc_t_stale = False

    def state_dict(self):
        return {"params": self.params, "m": self.m, "v": self.v, "step": self.step_t.cpu()}

    def load_state_dict(self, st):
        self.params.copy_(st["params"])
        self.m.copy_(st["m"])
        self.v.copy_(st["v"])
        self.step_t.fill_(int(st["step"][0]))
        self.refresh_shadow()
