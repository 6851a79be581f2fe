"""The C++ data-only pickle codec (csrc/bindings/pickle_native.cpp) against the reference
semantics in transport/serde_pickle.py: the same values, the same rejections, byte-identical
frames -- and the reference-wire ingestion no longer runs one Python opcode per tensor byte."""
import struct
import time

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from relayrl_prototype_amd import _native
from relayrl_prototype_amd.transport import serde_pickle as sp
from relayrl_prototype_amd.types import RelayRLAction


def _norm(v):
    """loads_fast's Vec<u8> bytearrays as lists of ints (what loads returns)."""
    if isinstance(v, bytearray):
        return list(v)
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_norm(x) for x in v)
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    return v


def _episode(n, rng, marker=True, dtype=np.float32, with_data=True):
    acts = []
    for i in range(n):
        data = {"logp_a": np.array([rng.normal()], np.float32), "v": np.array([rng.normal()], np.float32)} \
            if with_data else None
        acts.append(RelayRLAction(rng.normal(size=4).astype(dtype), np.array([i % 2], np.float32),
                                  np.ones(2, np.float32), float(rng.normal()), data, False, True))
    if marker:
        acts.append(RelayRLAction(None, None, None, 0.5, None, True, False))
    return acts


def _python_frame(actions):
    out = []
    for a in actions:
        d = a.to_json_dict()
        for key in ("obs", "act", "mask"):
            if d[key] is not None:
                d[key] = dict(d[key], data=list(d[key]["data"]))
        if d["data"] is not None:
            for k, v in d["data"].items():
                (kind, val), = v.items()
                if kind == "Tensor":
                    d["data"][k] = {"Tensor": dict(val, data=list(val["data"]))}
        out.append(d)
    return sp.dumps(out)


@pytest.mark.parametrize("n", [0, 1, 25, 300])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_native_writer_is_byte_identical(n, dtype):
    acts = _episode(n, np.random.default_rng(n), marker=n > 0, dtype=dtype)
    assert sp.reference_frame(acts) == _python_frame(acts)


def test_native_reader_matches_the_reference_interpreter():
    rng = np.random.default_rng(1)
    for n in (0, 1, 7, 120):
        f = sp.reference_frame(_episode(n, rng))
        ref = sp.loads(f)
        assert _native.pickle_loads(f, False) == ref
        assert _norm(sp.loads_fast(f)) == ref
        a_ref = sp.actions_from_reference(ref)
        a_fast = sp.actions_from_reference(sp.loads_fast(f))
        assert [x.to_json() for x in a_fast] == [x.to_json() for x in a_ref]


values = st.recursive(
    st.none() | st.booleans() | st.integers(-2 ** 70, 2 ** 70) | st.floats(allow_nan=False) | st.text(max_size=8)
    | st.binary(max_size=300),
    lambda ch: st.lists(ch, max_size=6) | st.tuples(ch, ch) | st.dictionaries(st.text(max_size=4), ch, max_size=4),
    max_leaves=30)


@settings(max_examples=200, deadline=None)
@given(values)
def test_roundtrip_of_arbitrary_data(v):
    f = _native.pickle_dumps(v)
    assert f == sp.dumps(v)
    assert _native.pickle_loads(f) == sp.loads(f)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.binary(min_size=1, max_size=64))
def test_garbage_is_rejected_like_the_reference(tail):
    f = b"\x80\x03" + tail
    try:
        ref = sp.loads(f)
    except Exception as e:  # noqa: BLE001
        ref = type(e)
    try:
        nat = _native.pickle_loads(f)
    except Exception as e:  # noqa: BLE001
        nat = type(e)
    if isinstance(ref, type):
        assert isinstance(nat, type), (f, ref, nat)
        assert issubclass(nat, ValueError) == issubclass(ref, ValueError), (f, ref, nat)
    else:
        assert nat == ref


@pytest.mark.parametrize("op", [b"c", b"\x93", b"R", b"b", b"i", b"o", b"\x81", b"\x92", b"\x82", b"P", b"Q"])
def test_code_execution_opcodes_are_rejected(op):
    with pytest.raises(ValueError):
        _native.pickle_loads(b"\x80\x03" + op + b"os\nsystem\n.")


def test_memo_and_marks():
    # memoised list referenced twice, tuples, sets, LONG1, BINFLOAT, nested marks
    f = (b"\x80\x03]q\x00(K\x01K\x02eh\x00\x86(\x8a\x02\x00\x01G?\xf0\x00\x00\x00\x00\x00\x00t\x8f(K\x05\x90\x87.")
    assert _native.pickle_loads(f) == sp.loads(f)
    assert _norm(_native.pickle_loads(f, True)) == sp.loads(f)


def test_native_decode_is_much_faster():
    f = sp.reference_frame(_episode(25, np.random.default_rng(3)))
    t0 = time.perf_counter()
    for _ in range(5):
        sp.loads(f)
    t_py = (time.perf_counter() - t0) / 5
    t0 = time.perf_counter()
    for _ in range(50):
        sp.loads_fast(f)
    t_nat = (time.perf_counter() - t0) / 50
    assert t_nat * 20 < t_py, (t_nat, t_py)
