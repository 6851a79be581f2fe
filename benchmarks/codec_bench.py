#!/usr/bin/env python3
"""Codec benchmarks (reference benches T2: rf/benches/runtime_benchmarks.rs, disabled there):
safetensors TensorData round trips for TENSOR_SIZES x dtypes, RRLT trajectory
encode/decode and reference-JSON action round trips."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

TENSOR_SIZES = [1, 10, 15, 25, 50, 100, 250, 500, 1000, 10000]
TRAJ_SIZES = [5, 10, 50, 100, 500, 1000, 5000, 10000]


def t(fn, n=200):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.types import RelayRLAction, RelayRLTrajectory

    res = {"tensor_roundtrip_us": {}, "traj_encode_us": {}, "traj_decode_us": {}}
    for dt, np_dt in (("Float", np.float32), ("Double", np.float64), ("Long", np.int64), ("Byte", np.uint8)):
        for n in TENSOR_SIZES:
            a = np.arange(n).astype(np_dt)
            res["tensor_roundtrip_us"][f"{dt}[{n}]"] = t(
                lambda: _native.st_decode(_native.st_encode(dt, [n], a.tobytes())))
    for n in TRAJ_SIZES:
        tr = RelayRLTrajectory(n + 1, None)
        for i in range(n):
            tr.add_action(RelayRLAction(obs=np.zeros(4, np.float32), act=np.array([1], np.int32),
                                        mask=np.ones(2, np.float32), rew=1.0, data={"logp_a": np.float32(-0.7)}))
        b = tr.encode()
        reps = max(3, 2000 // n)
        res["traj_encode_us"][n] = t(tr.encode, reps)
        res["traj_decode_us"][n] = t(lambda: RelayRLTrajectory.decode(b), reps)
        res.setdefault("traj_bytes_per_action", {})[n] = len(b) / n
    a = RelayRLAction(obs=np.zeros(4), act=np.array([1.0]), mask=np.ones(2), rew=1.0, data={"logp_a": np.float32(-1)})
    res["action_json_roundtrip_us"] = t(lambda: RelayRLAction.action_from_json(a.to_json()))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
