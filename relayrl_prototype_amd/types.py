"""RelayRLAction / RelayRLTrajectory (reference: rf/src/types/{action,trajectory}.rs and
their PyO3 classes o3_action.rs:48-235, o3_trajectory.rs:34-166).

Host-side record types of the agent API.  Tensors are kept as numpy arrays with their
dtype and shape (the reference flattened everything to f64 via tolist(), defect A12);
the wire encodings are native C++ (``_native``):

* ``TensorData`` JSON form = {"shape", "dtype", "data": bytes of a one-tensor
  safetensors file} -- byte-compatible with the reference (action.rs:342-352);
* trajectories travel as RRLT binary frames (``RelayRLTrajectory.encode``).

The on-GPU actor never builds these objects: it writes SoA rollout buffers in HBM.
"""
from __future__ import annotations

import json
import struct
import threading
from typing import Any, Dict, List, Optional

import numpy as np

from . import _native

_NP2DT = {
    np.dtype(np.uint8): "Byte",
    np.dtype(np.int16): "Short",
    np.dtype(np.int32): "Int",
    np.dtype(np.int64): "Long",
    np.dtype(np.float32): "Float",
    np.dtype(np.float64): "Double",
    np.dtype(np.bool_): "Bool",
}
_DT2NP = {v: k for k, v in _NP2DT.items()}
_SCALAR_KINDS = ("Byte", "Short", "Int", "Long", "Float", "Double", "String", "Bool")


def to_numpy(x) -> Optional[np.ndarray]:
    """numpy / torch / list / scalar -> contiguous numpy array with a supported dtype."""
    if x is None:
        return None
    if hasattr(x, "detach") and hasattr(x, "cpu"):  # torch.Tensor
        x = x.detach().cpu().numpy()
    a = np.asarray(x)
    if a.dtype not in _NP2DT:
        if np.issubdtype(a.dtype, np.floating):
            a = a.astype(np.float32)
        elif np.issubdtype(a.dtype, np.integer):
            a = a.astype(np.int64)
        else:
            raise TypeError(f"unsupported tensor dtype {a.dtype}")
    return np.ascontiguousarray(a)


def tensor_to_wire(a: np.ndarray):
    return (_NP2DT[a.dtype], list(a.shape), a.tobytes())


def tensor_from_wire(t) -> np.ndarray:
    dt, shape, raw = t
    return np.frombuffer(raw, dtype=_DT2NP[dt]).reshape(shape).copy()


def tensordata_json(a: np.ndarray) -> dict:
    """Reference TensorData serde form: data = one-tensor safetensors file as u8 list."""
    dt, shape, raw = tensor_to_wire(a)
    st = _native.st_encode(dt, shape, raw)
    return {"shape": shape, "dtype": dt, "data": list(st)}


def tensordata_from_json(d: dict) -> np.ndarray:
    dt, shape, raw = _native.st_decode(bytes(d["data"]))
    a = np.frombuffer(raw, dtype=_DT2NP[dt]).reshape(shape).copy()
    if d.get("dtype") == "Bool":
        a = a.astype(np.bool_)
    return a


def _aux_to_wire(v):
    if isinstance(v, (bool, np.bool_)):
        return ("Bool", bool(v))
    if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
        return ("Long", int(v))
    if isinstance(v, (float, np.floating)):
        return ("Double", float(v))
    if isinstance(v, str):
        return ("String", v)
    return ("Tensor", tensor_to_wire(to_numpy(v)))


def _aux_from_wire(kv):
    kind, val = kv
    if kind == "Tensor":
        return tensor_from_wire(val)
    return val


class RelayRLAction:
    """One (obs, act, mask, reward, aux data, done) record (action.rs:421-689)."""

    __slots__ = ("_obs", "_act", "_mask", "_rew", "_data", "_done", "_reward_updated")

    def __init__(self, obs=None, act=None, mask=None, rew: float = 0.0, data: Optional[Dict[str, Any]] = None,
                 done: bool = False, reward_updated: bool = False):
        self._obs = to_numpy(obs)
        self._act = to_numpy(act)
        self._mask = to_numpy(mask)
        self._rew = float(rew)
        self._data = None if data is None else {str(k): v for k, v in data.items()}
        self._done = bool(done)
        self._reward_updated = bool(reward_updated)

    @classmethod
    def _trusted(cls, obs, act, mask, data) -> "RelayRLAction":
        """A step's record from arrays already in canonical form (contiguous, supported dtypes:
        the agent's native step), without re-validating them -- request_for_action's fast path."""
        a = object.__new__(cls)
        a._obs, a._act, a._mask, a._rew, a._data = obs, act, mask, 0.0, data
        a._done = a._reward_updated = False
        return a

    # getters (o3_action.rs:96-160)
    def get_obs(self) -> Optional[np.ndarray]:
        return self._obs

    def get_act(self) -> Optional[np.ndarray]:
        return self._act

    def get_mask(self) -> Optional[np.ndarray]:
        return self._mask

    def get_rew(self) -> float:
        return self._rew

    def get_data(self) -> Dict[str, Any]:
        if self._data is None:
            return {}
        out = {}
        for k, v in self._data.items():
            out[k] = to_numpy(v) if not isinstance(v, (bool, int, float, str, np.number, np.bool_)) else v
        return out

    def get_done(self) -> bool:
        return self._done

    def get_reward_updated(self) -> bool:
        return self._reward_updated

    def update_reward(self, reward: float) -> None:
        self._rew = float(reward)
        self._reward_updated = True

    # wire forms ---------------------------------------------------------
    def to_wire(self) -> dict:
        return {
            "obs": None if self._obs is None else tensor_to_wire(self._obs),
            "act": None if self._act is None else tensor_to_wire(self._act),
            "mask": None if self._mask is None else tensor_to_wire(self._mask),
            "rew": self._rew,
            "data": None if self._data is None else {k: _aux_to_wire(v) for k, v in self._data.items()},
            "done": self._done,
            "reward_updated": self._reward_updated,
        }

    @classmethod
    def from_wire(cls, d: dict) -> "RelayRLAction":
        a = cls.__new__(cls)
        a._obs = None if d["obs"] is None else tensor_from_wire(d["obs"])
        a._act = None if d["act"] is None else tensor_from_wire(d["act"])
        a._mask = None if d["mask"] is None else tensor_from_wire(d["mask"])
        a._rew = float(d["rew"])
        a._data = None if d["data"] is None else {k: _aux_from_wire(v) for k, v in d["data"].items()}
        a._done = bool(d["done"])
        a._reward_updated = bool(d["reward_updated"])
        return a

    def to_json_dict(self) -> dict:
        def td(x):
            return None if x is None else tensordata_json(x)

        data = None
        if self._data is not None:
            data = {}
            for k, v in self._data.items():
                kind, val = _aux_to_wire(v)
                data[k] = {"Tensor": tensordata_json(tensor_from_wire(val))} if kind == "Tensor" else {kind: val}
        return {"obs": td(self._obs), "act": td(self._act), "mask": td(self._mask), "rew": self._rew, "data": data,
                "done": self._done, "reward_updated": self._reward_updated}

    def to_json(self) -> str:
        """Reference serde JSON (o3_action.rs:162-175)."""
        return json.dumps(self.to_json_dict())

    @staticmethod
    def action_from_json(d) -> "RelayRLAction":
        if isinstance(d, str):
            d = json.loads(d)

        def td(x):
            return None if x is None else tensordata_from_json(x)

        data = None
        if d.get("data") is not None:
            data = {}
            for k, v in d["data"].items():
                (kind, val), = v.items()
                data[k] = tensordata_from_json(val) if kind == "Tensor" else val
        return RelayRLAction(td(d.get("obs")), td(d.get("act")), td(d.get("mask")), d.get("rew", 0.0), data,
                             d.get("done", False), d.get("reward_updated", False))

    def __repr__(self):
        return (f"RelayRLAction(obs={None if self._obs is None else self._obs.shape}, act={self._act}, "
                f"rew={self._rew}, done={self._done})")


class _PushPool:
    """One long-lived PUSH socket per trajectory-server address (the reference opened a
    new zmq Context + socket for every send, trajectory.rs:69-90)."""

    _lock = threading.Lock()
    _socks: Dict[str, Any] = {}

    @classmethod
    def get(cls, addr: str):
        with cls._lock:
            s = cls._socks.get(addr)
            if s is None or s.closed():
                s = _native.ZmtpSocket(_native.SockType.PUSH)
                s.connect(addr)
                cls._socks[addr] = s
            return s


class RelayRLTrajectory:
    """Ordered list of actions for one agent (trajectory.rs:96-204).

    ``add_action`` sends the trajectory to ``trajectory_server`` when a ``done`` action
    arrives (if ``send_if_done``) and then CLEARS it -- the reference only cleared at
    ``len >= max_length`` which made every upload cumulative (defect A1).
    """

    def __init__(self, max_length: int = 1000, trajectory_server: Optional[str] = "tcp://127.0.0.1:5556",
                 agent_id: str = "", sender=None, send_if_done: bool = False):
        self.max_length = int(max_length)
        self.trajectory_server = trajectory_server
        self.agent_id = agent_id
        self.seq = 0
        self.actions: List[RelayRLAction] = []
        self._sender = sender
        self._send_if_done = send_if_done

    def get_actions(self) -> List[RelayRLAction]:
        return list(self.actions)

    def __len__(self):
        return len(self.actions)

    def add_action(self, action: RelayRLAction, send_if_done: Optional[bool] = None) -> bool:
        """Append; on a done action optionally ship the episode.  Returns True if sent."""
        self.actions.append(action)
        send = self._send_if_done if send_if_done is None else send_if_done
        sent = False
        if action.get_done():
            if send:
                self.send()
                sent = True
            if sent or len(self.actions) >= self.max_length:
                self.actions.clear()
        elif len(self.actions) >= self.max_length and send:
            # truncated episode: ship what we have (not done) and start a new segment
            self.send()
            self.actions.clear()
            sent = True
        return sent

    def send(self):
        payload = self.encode()
        self.seq += 1
        if self._sender is not None:
            self._sender(payload)
        elif self.trajectory_server:
            _PushPool.get(self.trajectory_server).send([payload], 10000)

    def clear(self):
        self.actions.clear()

    # encodings --------------------------------------------------------
    def encode(self) -> bytes:
        return _native.traj_encode({"server": self.trajectory_server or "", "max_length": self.max_length,
                                    "agent_id": self.agent_id, "seq": self.seq,
                                    "actions": [a.to_wire() for a in self.actions]})

    @staticmethod
    def decode(buf: bytes) -> "RelayRLTrajectory":
        d = _native.traj_decode(buf)
        t = RelayRLTrajectory(d["max_length"], d["server"] or None, d["agent_id"])
        t.seq = d["seq"]
        t.actions = [RelayRLAction.from_wire(a) for a in d["actions"]]
        return t

    def to_json(self) -> str:
        """{"inner": {trajectory_server, max_length, actions}} (o3_trajectory.rs:75-78)."""
        return json.dumps({"inner": {"trajectory_server": self.trajectory_server, "max_length": self.max_length,
                                     "actions": [a.to_json_dict() for a in self.actions]}})

    @staticmethod
    def traj_from_json(d) -> "RelayRLTrajectory":
        if isinstance(d, str):
            d = json.loads(d)
        inner = d["inner"] if "inner" in d else d
        t = RelayRLTrajectory(inner.get("max_length", 1000), inner.get("trajectory_server"))
        t.actions = [RelayRLAction.action_from_json(a) for a in inner.get("actions", [])]
        return t


# ---------------------------------------------------------------------- columnar episodes
_RRLC_MAGIC = b"RRLC"
_RRLC_HDR = "<4sIIIIIBBBBq"  # magic, version, n, D, K, A, act_kind, has_mask, has_logp, flags, seq
_ACT_KINDS = {0: np.float32, 1: np.int32}


class TrajectoryColumns:
    """One episode (or truncated segment) as columns -- the agent's fast upload format.

    The reference pickles a ``Vec<RelayRLAction>`` with one safetensors file per tensor
    (trajectory.rs:50-55, action.rs:40-90), i.e. O(actions x tensors) encode work on the
    agent and the learner.  An RRLC frame is a fixed header + agent id + contiguous
    little-endian arrays (obs [n,D] f32, act [n,K] f32|i32, mask [n,A] f32, rew [n] f32,
    logp [n] f32, done [n] u8, then -- flags bit 0 -- next_obs [D] f32: the observation that
    follows the last action of a cut segment, whose value bootstraps it, like the
    reference's finish_path(last_val), replay_buffer.py:48-79), so encode is a handful of memcpys and decode is zero-copy
    ``np.frombuffer`` views that the learner appends to its flat buffer in one slice
    assignment.  ``get_actions()`` materialises RelayRLAction objects for code that wants
    the reference's per-action view.
    """

    __slots__ = ("obs", "act", "mask", "rew", "logp", "done", "agent_id", "seq", "max_length", "trajectory_server",
                 "next_obs")

    def __init__(self, obs, act, rew, done, mask=None, logp=None, agent_id: str = "", seq: int = 0,
                 max_length: int = 1000, next_obs=None):
        self.obs = obs
        self.act = act
        self.rew = rew
        self.done = done
        self.mask = mask
        self.logp = logp
        self.agent_id = agent_id
        self.seq = seq
        self.max_length = max_length
        self.trajectory_server = None
        self.next_obs = next_obs  # [D] or None: s_T of a cut (not done) segment

    def __len__(self):
        return int(self.rew.shape[0])

    @staticmethod
    def _rows(a, n):
        a = np.asarray(a)
        if n:
            return a.reshape(n, -1)
        return a.reshape(0, a.shape[-1] if a.ndim > 1 else 0)

    def encode(self) -> bytes:
        n = len(self)
        obs = self._rows(np.ascontiguousarray(self.obs, np.float32), n)
        act = self._rows(self.act, n)
        kind = 1 if np.issubdtype(act.dtype, np.integer) else 0
        act = np.ascontiguousarray(act, _ACT_KINDS[kind])
        A = 0 if self.mask is None else self._rows(self.mask, n).shape[1]
        aid = self.agent_id.encode()
        nxt = None if self.next_obs is None else np.ascontiguousarray(self.next_obs, np.float32).reshape(-1)
        if nxt is not None and nxt.size != obs.shape[1]:
            raise ValueError(f"next_obs has {nxt.size} values, observations have {obs.shape[1]}")
        hdr = struct.pack(_RRLC_HDR, _RRLC_MAGIC, 1, n, obs.shape[1], act.shape[1], A, kind,
                          self.mask is not None, self.logp is not None, 1 if nxt is not None else 0, int(self.seq))
        parts = [hdr, struct.pack("<H", len(aid)), aid, obs.tobytes(), act.tobytes()]
        if self.mask is not None:
            parts.append(np.ascontiguousarray(self.mask, np.float32).tobytes())
        parts.append(np.ascontiguousarray(self.rew, np.float32).tobytes())
        if self.logp is not None:
            parts.append(np.ascontiguousarray(self.logp, np.float32).tobytes())
        parts.append(np.ascontiguousarray(self.done, np.uint8).tobytes())
        if nxt is not None:
            parts.append(nxt.tobytes())
        return b"".join(parts)

    @staticmethod
    def is_frame(buf) -> bool:
        return bytes(buf[:4]) == _RRLC_MAGIC

    @staticmethod
    def decode(buf) -> "TrajectoryColumns":
        mv = memoryview(buf)
        hs = struct.calcsize(_RRLC_HDR)
        if len(mv) < hs + 2:
            raise ValueError("RRLC frame too short")
        magic, ver, n, D, K, A, kind, has_mask, has_logp, flags, seq = struct.unpack_from(_RRLC_HDR, mv, 0)
        if magic != _RRLC_MAGIC or ver != 1 or kind not in _ACT_KINDS or flags & ~1:
            raise ValueError("not an RRLC v1 frame")
        has_next = bool(flags & 1)
        (alen,) = struct.unpack_from("<H", mv, hs)
        off = hs + 2
        aid = bytes(mv[off:off + alen]).decode()
        off += alen
        need = off + 4 * n * (D + K + (A if has_mask else 0) + 1 + (1 if has_logp else 0)) + n + \
            (4 * D if has_next else 0)
        if len(mv) != need:
            raise ValueError(f"RRLC frame size {len(mv)} != expected {need}")

        def take(count, dt, shape):
            nonlocal off
            a = np.frombuffer(mv, dt, count, off).reshape(shape)
            off += count * np.dtype(dt).itemsize
            return a

        obs = take(n * D, np.float32, (n, D))
        act = take(n * K, _ACT_KINDS[kind], (n, K))
        mask = take(n * A, np.float32, (n, A)) if has_mask else None
        rew = take(n, np.float32, (n,))
        logp = take(n, np.float32, (n,)) if has_logp else None
        done = take(n, np.uint8, (n,))
        nxt = take(D, np.float32, (D,)) if has_next else None
        return TrajectoryColumns(obs, act, rew, done, mask, logp, aid, seq, next_obs=nxt)

    def get_actions(self) -> List[RelayRLAction]:
        out = []
        for i in range(len(self)):
            data = None if self.logp is None else {"logp_a": np.float32(self.logp[i])}
            out.append(RelayRLAction(self.obs[i].copy(), self.act[i].copy(),
                                     None if self.mask is None else self.mask[i].copy(), float(self.rew[i]), data,
                                     bool(self.done[i]), True))
        return out

    def to_trajectory(self) -> RelayRLTrajectory:
        t = RelayRLTrajectory(self.max_length, None, agent_id=self.agent_id)
        t.seq = self.seq
        t.actions = self.get_actions()
        return t


class ReferenceColumns:
    """A reference agent's upload (serde_pickle(Vec<RelayRLAction>), trajectory.rs:50-90) decoded
    natively into float32 columns (csrc/bindings/pickle_native.cpp ``reference_columns``): the
    action rows, the reference's terminal markers (rows without an observation,
    agent_zmq.rs:605-610) kept in place as ``has_obs == 0``.  EpisodeIngest applies the
    per-action semantics of the actions path to whole runs of rows at once; ``get_actions()``
    materialises RelayRLAction objects for plugin algorithms that want them.  Reference
    uploads carry no agent identity (a new connection per upload)."""

    _COLS = ("n", "obs", "has_obs", "act", "has_act", "mask", "has_mask", "rew", "done", "logp", "has_logp", "v",
             "has_v")
    __slots__ = _COLS + ("agent_id", "seq", "trajectory_server")

    def __init__(self, cols: dict):
        for k in self._COLS:
            setattr(self, k, cols[k])
        self.agent_id = "reference-agent"  # the upload's connection carries no identity
        self.seq = 0
        self.trajectory_server = None

    @staticmethod
    def decode(frame: bytes) -> "ReferenceColumns":
        return ReferenceColumns(_native.reference_columns(bytes(frame)))

    def __len__(self):
        return int(self.n)

    def tail(self, start: int) -> "ReferenceColumns":
        """Rows [start, n) (the deduper strips a re-sent prefix)."""
        d = {}
        for k in self._COLS[1:]:
            a = getattr(self, k)
            d[k] = None if a is None else a[start:]
        d["n"] = max(0, int(self.n) - start)
        return ReferenceColumns(d)

    @property
    def actions(self) -> List["RelayRLAction"]:
        """RelayRLTrajectory's attribute view (materialised on each access)."""
        return self.get_actions()

    def to_trajectory(self) -> "RelayRLTrajectory":
        """The same rows as a per-action RelayRLTrajectory, terminal markers kept in place (the
        form the ZMQ endpoint's fallback path produces for a ragged reference frame)."""
        t = RelayRLTrajectory(max(len(self), 1), None, self.agent_id)
        t.actions = self.get_actions()
        return t

    def encode(self) -> bytes:
        """One RRLT frame (the multi-rank engine relay forwards uploads as frames)."""
        return self.to_trajectory().encode()

    def get_actions(self) -> List["RelayRLAction"]:
        out = []
        for i in range(len(self)):
            def row(a, h):
                return None if a is None or not h[i] else a[i].copy()

            data = None
            if self.has_logp[i] or self.has_v[i]:
                data = {}
                if self.has_logp[i]:
                    data["logp_a"] = np.float32(self.logp[i])
                if self.has_v[i]:
                    data["v"] = np.float32(self.v[i])
            out.append(RelayRLAction(row(self.obs, self.has_obs), row(self.act, self.has_act),
                                     row(self.mask, self.has_mask), float(self.rew[i]), data, bool(self.done[i]),
                                     False))
        return out


def as_reference_trajectory(traj) -> "RelayRLTrajectory":
    """Any upload as the reference's per-action layout, the form plugin algorithms iterate
    (REINFORCE.py:70-95): actions with ``done=False`` and their data, each episode closed by the
    terminal marker ``(None, None, None, last_val, done=True)`` (agent_zmq.rs:605-610).

    * RelayRLTrajectory (RRLT / protobuf / reference frames): unchanged;
    * ReferenceColumns: its rows, markers already in place;
    * TrajectoryColumns (our agents' RRLC): rows + a marker; the marker's reward is 0 (a
      terminal state has no future; a cut segment's V(s_T) is the plugin's to estimate --
      agents running a plugin's model send actions with the marker already valued)."""
    if isinstance(traj, RelayRLTrajectory):
        return traj
    if isinstance(traj, ReferenceColumns):
        return traj.to_trajectory()
    if isinstance(traj, TrajectoryColumns):
        acts = []
        for a in traj.get_actions():
            acts.append(RelayRLAction(a.get_obs(), a.get_act(), a.get_mask(), a.get_rew(), a.get_data(), False,
                                      True))
        if len(acts):
            acts.append(RelayRLAction(None, None, None, 0.0, None, True, False))
        t = RelayRLTrajectory(traj.max_length, None, agent_id=traj.agent_id)
        t.seq = traj.seq
        t.actions = acts
        return t
    return traj


class EpisodeRecorder:
    """Preallocated per-agent episode columns; one row written per ``request_for_action``."""

    def __init__(self, capacity: int):
        self.capacity = int(capacity)
        self.n = 0
        self._shapes = None
        self._sink = None

    def _alloc(self, obs, act, mask):
        c = self.capacity
        self.obs = np.zeros((c, obs.size), np.float32)
        self.act = np.zeros((c, max(1, act.size)), np.int32 if np.issubdtype(act.dtype, np.integer) else np.float32)
        self.mask = None if mask is None else np.zeros((c, mask.size), np.float32)
        self.rew = np.zeros(c, np.float32)
        self.logp = np.zeros(c, np.float32)
        self.val = np.full(c, np.nan, np.float32)  # V(s_t) when the policy has a value head (reference wire)
        self.done = np.zeros(c, np.uint8)
        self._shapes = (obs.size, act.size, act.dtype.kind, None if mask is None else mask.size)
        self._sink = None

    def sink(self, obs_size: int, discrete: bool, act_dim: int):
        """The columns as a native ``RowSink`` for ``NativePolicy.step_row`` (which writes one
        row per call from C++), allocated for these shapes as ``record`` would for the policy's
        actions (0-d int32 when discrete, [act_dim] float32 otherwise) and [act_dim] masks."""
        key = (obs_size, 1, "i", act_dim) if discrete else (obs_size, act_dim, "f", act_dim)
        if self._shapes != key:
            if self.n:
                raise ValueError("observation/action shapes changed within an episode")
            act = np.zeros((), np.int32) if discrete else np.zeros(act_dim, np.float32)
            self._alloc(np.empty(obs_size, np.float32), act, np.empty(act_dim, np.float32))
        if self._sink is None:
            self._sink = _native.RowSink(self.obs, self.act, self.mask, self.logp, self.val, self.rew, self.done)
        return self._sink

    def record(self, obs: np.ndarray, act: np.ndarray, mask, logp, val=None) -> None:
        key = (obs.size, act.size, act.dtype.kind, None if mask is None else mask.size)
        if self._shapes != key:
            if self.n:
                raise ValueError("observation/action shapes changed within an episode")
            self._alloc(obs, act, mask)
        i = self.n
        self.obs[i] = obs.reshape(-1)
        self.act[i] = act.reshape(-1)
        if self.mask is not None:
            self.mask[i] = mask.reshape(-1)
        self.rew[i] = 0.0
        self.logp[i] = 0.0 if logp is None else float(logp)
        self.val[i] = np.nan if val is None else float(val)
        self.done[i] = 0
        self.n = i + 1

    def set_last_reward(self, r: float) -> None:
        if self.n:
            self.rew[self.n - 1] = r

    def full(self) -> bool:
        return self.n >= self.capacity

    def take(self, agent_id: str, seq: int, done: bool, next_obs=None) -> TrajectoryColumns:
        n = self.n
        d = self.done[:n].copy()
        if n and done:
            d[n - 1] = 1
        nxt = None if (done or next_obs is None) else np.asarray(next_obs, np.float32).reshape(-1).copy()
        cols = TrajectoryColumns(self.obs[:n].copy(), self.act[:n].copy(), self.rew[:n].copy(), d,
                                 None if self.mask is None else self.mask[:n].copy(), self.logp[:n].copy(),
                                 agent_id, seq, next_obs=nxt)
        self.n = 0
        return cols
