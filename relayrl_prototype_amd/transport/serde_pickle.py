"""Reference ZMQ trajectory frames: the ``serde_pickle`` encoding of ``Vec<RelayRLAction>``.

A reference agent uploads every finished episode as ``serde_pickle::to_writer(&actions)``
(trajectory.rs:50-55, decoded by training_zmq.rs:994-1012 with ``pickle::from_slice``).
serde_pickle writes a pickle protocol-3 stream of plain containers: a struct is a dict keyed
by field names, ``Option::None`` is ``None``, ``Vec<u8>`` a list of ints, a newtype enum
variant ``{name: value}`` (or ``(name, value)`` with its compat representation) and a unit
variant its name.

``loads`` here is NOT Python's unpickler: it is a small interpreter of the data-only opcode
subset (containers, scalars, strings, bytes, memo).  Every opcode that can import a name or
call one -- GLOBAL, STACK_GLOBAL, REDUCE, BUILD, INST, OBJ, NEWOBJ, EXT*, PERSID -- is an
error, so a frame can never execute anything.  ``dumps`` writes the same subset the way
serde_pickle does (protocol 3, no memo); tests use it to build reference-shaped fixtures.

``loads_fast`` / ``reference_frame`` run the same interpreter / writer in C++
(csrc/bindings/pickle_native.cpp, ~100x faster: the Python interpreter executes one opcode
per safetensors byte), Vec<u8> lists coming back as ``bytearray``; ``loads`` / ``dumps`` stay
the reference semantics the native codec is tested against (tests/test_pickle_native.py).

``actions_from_reference`` maps the decoded list onto :class:`RelayRLAction`s (TensorData =
{shape, dtype, data: bytes of a one-tensor safetensors file}, action.rs:193-352), and
:class:`CumulativeDeduper` strips the prefix a reference agent re-sends with every upload
(it never clears its trajectory below max_length: defect A1).
"""
from __future__ import annotations

import hashlib
import struct
from collections import OrderedDict
from typing import Any, List, Tuple

import numpy as np

MAX_DEPTH = 64
MAX_STACK = 1 << 20   # values on the interpreter stack (a frame holds ~10 per action)
MAX_MEMO = 1 << 16


class PickleFrameError(ValueError):
    pass


_MARK = object()


def is_pickle_frame(buf: bytes) -> bool:
    return len(buf) >= 2 and buf[0] == 0x80 and buf[1] <= 5


def loads(buf: bytes) -> Any:
    """Decode a data-only pickle (protocols 2-5 opcode subset); raises PickleFrameError on
    any opcode outside the subset and on any malformed frame."""
    try:
        return _loads(buf)
    except (IndexError, KeyError, TypeError) as e:  # e.g. BINPUT on an empty stack, BINGET of an unknown key
        raise PickleFrameError(f"malformed frame: {type(e).__name__}") from None


def _loads(buf: bytes) -> Any:
    mv = memoryview(buf)
    n = len(mv)
    pos = 0
    stack: List[Any] = []
    memo = {}
    marks = 0  # MARKs on the stack (a running count: O(1) per MARK / pop_mark)

    def take(k: int) -> memoryview:
        nonlocal pos
        if pos + k > n:
            raise PickleFrameError("truncated frame")
        out = mv[pos:pos + k]
        pos += k
        return out

    def pop_mark() -> List[Any]:
        nonlocal marks
        if marks == 0:
            raise PickleFrameError("MARK not found")
        for i in range(len(stack) - 1, -1, -1):
            if stack[i] is _MARK:
                items = stack[i + 1:]
                del stack[i:]
                marks -= 1
                return items
        raise PickleFrameError("MARK not found")

    def pop_value():
        if not stack or stack[-1] is _MARK:
            raise PickleFrameError("stack underflow")
        return stack.pop()

    def top_container(kind):
        if not stack or not isinstance(stack[-1], kind):
            raise PickleFrameError(f"expected a {kind.__name__} on the stack")
        return stack[-1]

    while True:
        if len(stack) > MAX_STACK or len(memo) > MAX_MEMO:
            raise PickleFrameError("frame too large")
        op = take(1)[0]
        if op == 0x80:  # PROTO
            take(1)
        elif op == 0x95:  # FRAME
            take(8)
        elif op == 0x2E:  # STOP
            if len(stack) != 1:
                raise PickleFrameError("bad stack at STOP")
            return stack[0]
        elif op == 0x4E:  # NONE
            stack.append(None)
        elif op == 0x88:
            stack.append(True)
        elif op == 0x89:
            stack.append(False)
        elif op == 0x4B:  # BININT1
            stack.append(take(1)[0])
        elif op == 0x4D:  # BININT2
            stack.append(struct.unpack("<H", take(2))[0])
        elif op == 0x4A:  # BININT
            stack.append(struct.unpack("<i", take(4))[0])
        elif op == 0x8A:  # LONG1
            k = take(1)[0]
            stack.append(int.from_bytes(take(k), "little", signed=True) if k else 0)
        elif op == 0x8B:  # LONG4
            k = struct.unpack("<i", take(4))[0]
            if k < 0 or k > 64:
                raise PickleFrameError("LONG4 too large")
            stack.append(int.from_bytes(take(k), "little", signed=True) if k else 0)
        elif op == 0x47:  # BINFLOAT (big-endian double)
            stack.append(struct.unpack(">d", take(8))[0])
        elif op == 0x58:  # BINUNICODE
            k = struct.unpack("<I", take(4))[0]
            stack.append(str(take(k), "utf-8"))
        elif op == 0x8C:  # SHORT_BINUNICODE
            k = take(1)[0]
            stack.append(str(take(k), "utf-8"))
        elif op == 0x8D:  # BINUNICODE8
            k = struct.unpack("<Q", take(8))[0]
            stack.append(str(take(k), "utf-8"))
        elif op == 0x42:  # BINBYTES
            k = struct.unpack("<I", take(4))[0]
            stack.append(bytes(take(k)))
        elif op == 0x43:  # SHORT_BINBYTES
            k = take(1)[0]
            stack.append(bytes(take(k)))
        elif op == 0x8E:  # BINBYTES8
            k = struct.unpack("<Q", take(8))[0]
            stack.append(bytes(take(k)))
        elif op == 0x28:  # MARK
            if marks >= MAX_DEPTH:
                raise PickleFrameError("nesting too deep")
            stack.append(_MARK)
            marks += 1
        elif op == 0x5D:  # EMPTY_LIST
            stack.append([])
        elif op == 0x7D:  # EMPTY_DICT
            stack.append({})
        elif op == 0x29:  # EMPTY_TUPLE
            stack.append(())
        elif op == 0x8F:  # EMPTY_SET
            stack.append(set())
        elif op == 0x61:  # APPEND
            v = pop_value()
            top_container(list).append(v)
        elif op == 0x65:  # APPENDS
            items = pop_mark()
            top_container(list).extend(items)
        elif op == 0x73:  # SETITEM
            v = pop_value()
            k = pop_value()
            top_container(dict)[_key(k)] = v
        elif op == 0x75:  # SETITEMS
            items = pop_mark()
            if len(items) % 2:
                raise PickleFrameError("odd SETITEMS")
            d = top_container(dict)
            for i in range(0, len(items), 2):
                d[_key(items[i])] = items[i + 1]
        elif op == 0x90:  # ADDITEMS
            items = pop_mark()
            top_container(set).update(_key(x) for x in items)
        elif op == 0x91:  # FROZENSET
            stack.append(frozenset(_key(x) for x in pop_mark()))
        elif op == 0x74:  # TUPLE
            stack.append(tuple(pop_mark()))
        elif op in (0x85, 0x86, 0x87):  # TUPLE1..3
            k = op - 0x84
            if len(stack) < k:
                raise PickleFrameError("stack underflow")
            items = stack[-k:]
            del stack[-k:]
            stack.append(tuple(items))
        elif op == 0x71:  # BINPUT
            memo[take(1)[0]] = stack[-1]
        elif op == 0x72:  # LONG_BINPUT
            memo[struct.unpack("<I", take(4))[0]] = stack[-1]
        elif op == 0x94:  # MEMOIZE
            memo[len(memo)] = stack[-1]
        elif op == 0x68:  # BINGET
            stack.append(memo[take(1)[0]])
        elif op == 0x6A:  # LONG_BINGET
            stack.append(memo[struct.unpack("<I", take(4))[0]])
        elif op == 0x30:  # POP
            if not stack:
                raise PickleFrameError("stack underflow")
            if stack.pop() is _MARK:
                marks -= 1
        elif op == 0x31:  # POP_MARK
            pop_mark()
        else:
            raise PickleFrameError(f"opcode 0x{op:02x} is not allowed in a trajectory frame")


def loads_fast(buf: bytes) -> Any:
    """``loads`` in C++, lists of u8 (serde's Vec<u8>) as ``bytearray`` (so an EMPTY list of
    any type is an empty bytearray; the consumers below accept both)."""
    try:
        from .. import _native
    except ImportError:  # the host runtime is not built: the reference interpreter
        return loads(buf)
    try:
        return _native.pickle_loads(bytes(buf), True)
    except _native.PickleFrameError as e:
        raise PickleFrameError(str(e)) from None


def _seq(v) -> list:
    """A decoded sequence (list, tuple, or a Vec<u8> bytearray from loads_fast) as a list."""
    return list(v)


def _key(k):
    if isinstance(k, (list, dict, set)):
        raise PickleFrameError("unhashable key")
    return k


# ---------------------------------------------------------------------- writer (serde_pickle style)
def dumps(obj: Any) -> bytes:
    out = bytearray(b"\x80\x03")
    _dump(obj, out, 0)
    out += b"."
    return bytes(out)


def _dump(o: Any, out: bytearray, depth: int):
    if depth > MAX_DEPTH:
        raise ValueError("nesting too deep")
    if o is None:
        out += b"N"
    elif o is True:
        out += b"\x88"
    elif o is False:
        out += b"\x89"
    elif isinstance(o, int):
        if 0 <= o < 256:
            out += b"K" + bytes([o])
        elif 0 <= o < 65536:
            out += b"M" + struct.pack("<H", o)
        elif -2**31 <= o < 2**31:
            out += b"J" + struct.pack("<i", o)
        else:
            raw = o.to_bytes((o.bit_length() + 8) // 8, "little", signed=True)
            out += b"\x8a" + bytes([len(raw)]) + raw
    elif isinstance(o, float):
        out += b"G" + struct.pack(">d", o)
    elif isinstance(o, str):
        raw = o.encode("utf-8")
        out += b"X" + struct.pack("<I", len(raw)) + raw
    elif isinstance(o, (bytes, bytearray)):
        out += (b"C" + bytes([len(o)]) if len(o) < 256 else b"B" + struct.pack("<I", len(o))) + bytes(o)
    elif isinstance(o, tuple):
        if len(o) == 0:
            out += b")"
        else:
            out += b"("
            for x in o:
                _dump(x, out, depth + 1)
            out += b"t"
    elif isinstance(o, list):
        out += b"]"
        for i in range(0, len(o), 1000):
            out += b"("
            for x in o[i:i + 1000]:
                _dump(x, out, depth + 1)
            out += b"e"
    elif isinstance(o, dict):
        out += b"}"
        if o:
            out += b"("
            for k, v in o.items():
                _dump(k, out, depth + 1)
                _dump(v, out, depth + 1)
            out += b"u"
    else:
        raise TypeError(f"cannot serialise {type(o).__name__}")


# ---------------------------------------------------------------------- reference actions
def enum_variant(v: Any) -> Tuple[str, Any]:
    """serde enum in any serde_pickle representation -> (variant, payload)."""
    if isinstance(v, str):
        return v, None
    if isinstance(v, dict) and len(v) == 1:
        (k, val), = v.items()
        return str(k), val
    if isinstance(v, (tuple, list)) and 1 <= len(v) <= 2 and isinstance(v[0], str):
        return v[0], (v[1] if len(v) == 2 else None)
    raise PickleFrameError(f"not an enum value: {type(v).__name__}")


def _tensordata(d: Any):
    from ..types import tensordata_from_json

    if d is None:
        return None
    if not isinstance(d, dict) or "data" not in d:
        raise PickleFrameError("TensorData must be a dict with shape / dtype / data")
    dt, _ = enum_variant(d.get("dtype", "Float"))
    data = d["data"]
    raw = bytes(data) if isinstance(data, (bytes, bytearray, list, tuple)) else None
    if raw is None:
        raise PickleFrameError("TensorData.data must be bytes or a list of u8")
    return tensordata_from_json({"shape": _seq(d.get("shape", [])), "dtype": dt, "data": raw})


def actions_from_reference(obj: Any):
    """Decoded ``Vec<RelayRLAction>`` (or a RelayRLTrajectory struct) -> [RelayRLAction]."""
    from ..types import RelayRLAction

    if isinstance(obj, dict) and "actions" in obj:  # a whole RelayRLTrajectory struct
        obj = obj["actions"]
    if isinstance(obj, bytearray) and not obj:  # loads_fast: an empty list
        obj = []
    if not isinstance(obj, (list, tuple)):
        raise PickleFrameError("expected a list of actions")
    out = []
    for a in obj:
        if not isinstance(a, dict):
            raise PickleFrameError("an action must be a dict")
        data = None
        if a.get("data") is not None:
            data = {}
            for k, v in a["data"].items():
                kind, val = enum_variant(v)
                data[str(k)] = _tensordata(val) if kind == "Tensor" else val
        out.append(RelayRLAction(_tensordata(a.get("obs")), _tensordata(a.get("act")), _tensordata(a.get("mask")),
                                 float(a.get("rew", 0.0)), data, bool(a.get("done", False)),
                                 bool(a.get("reward_updated", False))))
    return out


def reference_frame(actions) -> bytes:
    """[RelayRLAction] -> the frame a reference agent would send (serde_pickle of the
    actions' serde form; enums in serde_pickle's default ``{variant: value}`` / name form;
    TensorData.data as a list of u8).  Written by the C++ writer when the host runtime is
    built (bytes as Vec<u8> lists), else by ``dumps``: byte-identical output."""
    out = [a.to_json_dict() for a in actions]
    try:
        from .. import _native

        return _native.pickle_dumps(out, True)
    except ImportError:
        pass
    for d in out:
        for key in ("obs", "act", "mask"):
            if d[key] is not None:
                d[key] = dict(d[key], data=list(d[key]["data"]))
        if d["data"] is not None:
            for k, v in d["data"].items():
                (kind, val), = v.items()
                if kind == "Tensor":
                    d["data"][k] = {"Tensor": dict(val, data=list(val["data"]))}
    return dumps(out)


class ReferenceDeduper:
    """Reference agents re-send every earlier episode with each upload (the trajectory is
    only cleared at max_length, trajectory.rs:160-204), each over a NEW connection, so the
    learner would train on the same actions again and again.  Uploads are matched by a
    digest of their first row.  An upload keeps only its new rows when it strictly extends a
    remembered upload AT AN EPISODE BOUNDARY: the remembered prefix must end in a ``done``
    row, which every cumulative re-send does (the agent sends right after appending a done
    marker, trajectory.rs:172-203).

    One deduper serves both decode paths of the ZMQ endpoint -- natively decoded columns
    (``new_rows``, types.ReferenceColumns) and per-action objects (``new_actions``, the path
    for ragged frames) -- with ONE digest definition over a canonical row encoding
    (``flag, f32 obs | flag, f32 act | f32 rew, u8 done``), so an agent whose first upload went
    one way and whose re-send goes the other is still stripped.

    Residual ambiguity: the sender is not part of the key -- each reference upload comes
    over a fresh PUSH connection with no identity, so two agents cannot be told apart.  An
    upload of the same length as a remembered one is therefore never dropped: the
    reference never re-sends an upload unchanged (every send follows a new done action),
    while two identical independent episodes (deterministic policy, fixed start state) are
    real data.  Only an independent episode that begins with another complete episode's
    exact action sequence would still be trimmed."""

    def __init__(self, capacity: int = 4096):
        self.capacity = capacity
        self._seen: "OrderedDict[bytes, Tuple[int, bytes]]" = OrderedDict()
        self.stripped = 0

    # canonical row bytes ------------------------------------------------------------
    @staticmethod
    def _row_bytes(a) -> bytes:
        out = []
        for t in (a.get_obs(), a.get_act()):
            if t is None:
                out.append(b"\x00")
            else:
                out.append(b"\x01" + np.ascontiguousarray(np.asarray(t, np.float32).reshape(-1)).tobytes())
        out.append(struct.pack("<fB", float(a.get_rew()), 1 if a.get_done() else 0))
        return b"".join(out)

    @staticmethod
    def _digest_actions(actions) -> bytes:
        h = hashlib.blake2b(digest_size=16)
        for a in actions:
            h.update(ReferenceDeduper._row_bytes(a))
        return h.digest()

    @staticmethod
    def _digest_cols(c, k: int) -> bytes:
        """The same byte stream as ``_digest_actions`` over rows [0, k), built per run of rows
        with the same (has_obs, has_act) pattern as one fixed-width byte matrix."""
        h = hashlib.blake2b(digest_size=16)
        ho = np.asarray(c.has_obs[:k], bool)
        ha = np.asarray(c.has_act[:k], bool)
        pat = ho.astype(np.int8) * 2 + ha.astype(np.int8)
        cuts = np.flatnonzero(np.diff(pat)) + 1
        starts = np.concatenate(([0], cuts)).astype(int)
        ends = np.concatenate((cuts, [k])).astype(int)
        rew = np.asarray(c.rew, np.float32)
        done = np.asarray(c.done).astype(np.uint8)
        for s0, e0 in zip(starts, ends):
            if e0 <= s0:
                continue
            parts = []
            n = e0 - s0
            for has, arr in ((ho[s0], c.obs), (ha[s0], c.act)):
                if has:
                    parts.append(np.ones((n, 1), np.uint8))
                    parts.append(np.ascontiguousarray(np.asarray(arr[s0:e0], np.float32).reshape(n, -1)).view(np.uint8))
                else:
                    parts.append(np.zeros((n, 1), np.uint8))
            parts.append(rew[s0:e0].reshape(n, 1).view(np.uint8))
            parts.append(done[s0:e0].reshape(n, 1))
            h.update(np.concatenate(parts, axis=1).tobytes())
        return h.digest()

    # the shared rule -----------------------------------------------------------------
    def _keep_from(self, n: int, head: bytes, prefix_digest, full_digest, done_at) -> int:
        """Index of the first row to keep (0 = keep all), updating the memory."""
        start = 0
        prev = self._seen.get(head)
        if prev is not None:
            n_prev, dig = prev
            if n > n_prev and done_at(n_prev - 1) and prefix_digest(n_prev) == dig:
                start = n_prev
                self.stripped += n_prev
        self._seen[head] = (n, full_digest())
        self._seen.move_to_end(head)
        while len(self._seen) > self.capacity:
            self._seen.popitem(last=False)
        return start

    def new_rows(self, c):
        n = len(c)
        if n == 0:
            return c
        start = self._keep_from(n, self._digest_cols(c, 1), lambda k: self._digest_cols(c, k),
                                lambda: self._digest_cols(c, n), lambda i: bool(c.done[i]))
        return c.tail(start) if start else c

    def new_actions(self, actions) -> list:
        if not actions:
            return actions
        n = len(actions)
        start = self._keep_from(n, self._digest_actions(actions[:1]), lambda k: self._digest_actions(actions[:k]),
                                lambda: self._digest_actions(actions), lambda i: bool(actions[i].get_done()))
        return actions[start:] if start else actions


# the two decode paths' historical names: one class, one digest
ColumnDeduper = ReferenceDeduper
CumulativeDeduper = ReferenceDeduper
