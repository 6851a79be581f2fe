"""gRPC transport: the ``relayrl_grpc.RelayRLRoute`` service of rf/proto/relayrl_grpc.proto.

``protoc`` / ``grpc_tools`` are not installed, so the message classes are built at import
time from a hand-written FileDescriptorProto with the exact field numbers and types of
the reference proto (wire-compatible with tonic clients):

  RelayRLAction{bytes obs=1, action=2, mask=3; float reward=4; map<string,bytes> data=5;
                bool done=6, reward_update_flag=7}
  Trajectory{repeated RelayRLAction actions=1}
  RelayRLModel{int32 code=1; bytes model=2; int64 version=3; string error=4}
  RequestModel{int32 first_time=1; int64 version=2}
  ActionResponse{int32 code=1; string message=2}
  service RelayRLRoute{ SendActions(Trajectory) -> ActionResponse;
                        ClientPoll(RequestModel) -> RelayRLModel }

Tensor fields carry one-tensor safetensors files, ``data`` values carry the JSON of the
RelayRLData enum (grpc_utils.rs:31-129).  Fixes vs the reference: real model versions
(A5), no tempfile round trip for models (grpc_utils.rs:171-205), no process::exit on an
RPC error (agent_grpc.rs:528-531), bounded connect retries (A4).
Extensions (reference tonic clients never call them, so wire compatibility holds):
``first_time & 2`` asks for RRLM flat-weight frames instead of a TorchScript archive, and
``SendFrame(TrajectoryFrame{bytes frame=1})`` uploads one columnar RRLC / RRLT episode
frame instead of a per-action protobuf (one memcpy-sized message per episode).  The
agent keeps a background long-poll thread for model updates, so an upload never waits
on ``ClientPoll`` (the reference polled synchronously after every send, agent_grpc.rs).

``ReferenceGrpcAgentTransport`` is the reference agent's OWN gRPC dialect, to train against a
reference (tonic) training server: ``ClientPoll{first_time: 1, version: 0}`` every 500 ms
until a TorchScript archive arrives, per-episode ``SendActions`` with safetensors tensor
fields / JSON ``RelayRLData`` / ``reward_update_flag = false``, then one synchronous
``ClientPoll{first_time: 0, version}`` that swaps the policy on a non-empty model.
"""
from __future__ import annotations

import json
import threading
import time
from concurrent import futures
from typing import Callable, Optional

import numpy as np

from ..runtime.model_store import ModelBlob
from ..types import RelayRLAction, RelayRLTrajectory, tensordata_from_json, to_numpy

_PKG = "relayrl_grpc"


def _build_messages():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="relayrl_grpc.proto", package=_PKG, syntax="proto3")

    def msg(name, fields, nested=None):
        m = fdp.message_type.add(name=name)
        for fname, num, ftype, label, type_name in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if type_name:
                f.type_name = type_name
        if nested:
            nested(m)
        return m

    OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

    def data_entry(m):
        e = m.nested_type.add(name="DataEntry")
        e.field.add(name="key", number=1, type=F.TYPE_STRING, label=OPT)
        e.field.add(name="value", number=2, type=F.TYPE_BYTES, label=OPT)
        e.options.map_entry = True

    msg("RelayRLAction", [("obs", 1, F.TYPE_BYTES, OPT, None), ("action", 2, F.TYPE_BYTES, OPT, None),
                          ("mask", 3, F.TYPE_BYTES, OPT, None), ("reward", 4, F.TYPE_FLOAT, OPT, None),
                          ("data", 5, F.TYPE_MESSAGE, REP, f".{_PKG}.RelayRLAction.DataEntry"),
                          ("done", 6, F.TYPE_BOOL, OPT, None), ("reward_update_flag", 7, F.TYPE_BOOL, OPT, None)],
        data_entry)
    msg("Trajectory", [("actions", 1, F.TYPE_MESSAGE, REP, f".{_PKG}.RelayRLAction")])
    msg("RelayRLModel", [("code", 1, F.TYPE_INT32, OPT, None), ("model", 2, F.TYPE_BYTES, OPT, None),
                         ("version", 3, F.TYPE_INT64, OPT, None), ("error", 4, F.TYPE_STRING, OPT, None)])
    msg("RequestModel", [("first_time", 1, F.TYPE_INT32, OPT, None), ("version", 2, F.TYPE_INT64, OPT, None)])
    msg("TrajectoryFrame", [("frame", 1, F.TYPE_BYTES, OPT, None)])
    msg("ActionResponse", [("code", 1, F.TYPE_INT32, OPT, None), ("message", 2, F.TYPE_STRING, OPT, None)])
    svc = fdp.service.add(name="RelayRLRoute")
    svc.method.add(name="SendActions", input_type=f".{_PKG}.Trajectory", output_type=f".{_PKG}.ActionResponse")
    svc.method.add(name="SendFrame", input_type=f".{_PKG}.TrajectoryFrame", output_type=f".{_PKG}.ActionResponse")
    svc.method.add(name="ClientPoll", input_type=f".{_PKG}.RequestModel", output_type=f".{_PKG}.RelayRLModel")
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    get = message_factory.GetMessageClass
    return {n: get(pool.FindMessageTypeByName(f"{_PKG}.{n}"))
            for n in ("RelayRLAction", "Trajectory", "RelayRLModel", "RequestModel", "ActionResponse",
                      "TrajectoryFrame")}, fdp


MESSAGES, FILE_DESCRIPTOR = _build_messages()
PbAction = MESSAGES["RelayRLAction"]
PbTrajectory = MESSAGES["Trajectory"]
PbModel = MESSAGES["RelayRLModel"]
PbRequest = MESSAGES["RequestModel"]
PbResponse = MESSAGES["ActionResponse"]
PbFrame = MESSAGES["TrajectoryFrame"]
SERVICE = f"{_PKG}.RelayRLRoute"


# ---------------------------------------------------------------------- conversions
def _st(a) -> bytes:
    from ..types import tensor_to_wire
    from .. import _native

    dt, shape, raw = tensor_to_wire(to_numpy(a))
    return _native.st_encode(dt, shape, raw)


def _unst(b: bytes):
    from .. import _native
    from ..types import tensor_from_wire

    return tensor_from_wire(_native.st_decode(b))


def action_to_pb(a: RelayRLAction):
    """grpc_utils.rs:31-66 (reward_update_flag is carried, not hard-coded false)."""
    m = PbAction(reward=a.get_rew(), done=a.get_done(), reward_update_flag=a.get_reward_updated())
    if a.get_obs() is not None:
        m.obs = _st(a.get_obs())
    if a.get_act() is not None:
        m.action = _st(a.get_act())
    if a.get_mask() is not None:
        m.mask = _st(a.get_mask())
    d = a.to_json_dict().get("data") or {}
    for k, v in d.items():
        m.data[k] = json.dumps(v).encode()
    return m


def action_from_pb(m) -> RelayRLAction:
    data = None
    if len(m.data):
        data = {}
        for k, v in m.data.items():
            (kind, val), = json.loads(v.decode()).items()
            data[k] = tensordata_from_json(val) if kind == "Tensor" else val
    return RelayRLAction(_unst(m.obs) if m.obs else None, _unst(m.action) if m.action else None,
                         _unst(m.mask) if m.mask else None, m.reward, data, m.done, m.reward_update_flag)


def trajectory_to_pb(t: RelayRLTrajectory):
    return PbTrajectory(actions=[action_to_pb(a) for a in t.get_actions()])


def trajectory_from_pb(m, max_length: int = 1000) -> RelayRLTrajectory:
    t = RelayRLTrajectory(max_length, None)
    t.actions = [action_from_pb(a) for a in m.actions]
    return t


# ---------------------------------------------------------------------- server
def GrpcTrainingEndpoint(service, address: str, idle_timeout_ms: int = 30, native: Optional[bool] = None, **kw):
    """The RelayRLRoute server: the native one (C++ HTTP/2, csrc/net/h2grpc.cpp) when its module
    loads, else grpc.aio.  ``native=True`` requires it, ``False`` forces grpc.aio;
    RRL_GRPC_NATIVE=0 does the latter too."""
    from .h2_native import ERROR, load

    mod = load() if native is not False else None
    if mod is not None:
        return NativeGrpcTrainingEndpoint(service, address, idle_timeout_ms, mod, **kw)
    if native:
        from . import h2_native

        raise RuntimeError(f"native gRPC server unavailable: {h2_native.ERROR}")
    if native is None and ERROR is not None and "RRL_GRPC_NATIVE" not in ERROR:
        print(f"[grpc] native server unavailable ({ERROR}); serving with grpc.aio", flush=True)
    return AioGrpcTrainingEndpoint(service, address, idle_timeout_ms, **kw)


class NativeGrpcTrainingEndpoint:
    """RelayRLRoute on the native server: every RPC is parsed, queued and answered in C++ on one
    epoll thread (h2grpc.cpp); Python only consumes the queued uploads here -- one thread,
    decode + ``service.submit`` -- and hands each new model version to the server's model cell
    from a publisher thread (newest-wins).  A TorchScript archive a reference-dialect poll needs
    is built here on request (``NEED_TS``), once per version."""

    def __init__(self, service, address: str, idle_timeout_ms: int, mod, max_inbox: int = 65536,
                 max_inbox_bytes: int = 1 << 30, **_ignored):
        from ..runtime.model_store import LatestWorker

        self.service = service
        self._mod = mod
        addr = address.replace("tcp://", "")
        host, port = addr.rsplit(":", 1)
        if host in ("*", ""):
            host = "0.0.0.0"
        self.server = mod.GrpcServer(host, int(port), max_inbox, max_inbox_bytes, max(0, int(idle_timeout_ms)))
        self.port = self.server.port
        self.bad_frames = 0
        self.rejected = 0
        self._stop = threading.Event()
        blob = service.store.latest()
        if blob is not None:
            self._set_model(blob)
        self._publisher = LatestWorker(self._set_model, name="rrl-grpc-publisher")
        service.store.subscribe(self._publisher)
        self._thread = threading.Thread(target=self._consume, name="rrl-grpc-consumer", daemon=True)
        self._thread.start()

    def _set_model(self, blob):
        self.server.set_model(int(blob.version), blob.encode(), blob._ts)

    def _consume(self):
        from ..types import TrajectoryColumns

        mod = self._mod
        while not self._stop.is_set():
            it = self.server.recv(100)
            if it is None:
                continue
            kind, body, aux = it
            try:
                if kind == mod.NEED_TS:
                    blob = self.service.store.latest()
                    if blob is not None and blob.version == aux:
                        self.server.set_model_ts(aux, blob.torchscript())
                    continue
                if kind == mod.ACTIONS:
                    traj = trajectory_from_pb(PbTrajectory.FromString(body))
                    traj.agent_id = ""
                else:
                    traj = TrajectoryColumns.decode(body) if TrajectoryColumns.is_frame(body) else \
                        RelayRLTrajectory.decode(body)
            except Exception as e:  # noqa: BLE001 -- a bad upload is counted, the server keeps serving
                self.bad_frames += 1
                print(f"[grpc] bad upload: {e!r}", flush=True)
                continue
            self.service.submit(traj)  # blocking: a full learner queue parks the uploads in C++

    def flush(self, timeout_s: float = 10.0) -> bool:
        return self._publisher.flush(timeout_s)

    def stats(self) -> dict:
        return self.server.stats()

    def close(self, grace: float = 0.5):
        self.service.store.unsubscribe(self._publisher)
        self._publisher.close()
        self._stop.set()
        self._thread.join(timeout=5)
        self.server.close()


class AioGrpcTrainingEndpoint:
    """The RelayRLRoute server on ``grpc.aio``: one event-loop thread serves every RPC.

    The thread-pool server (round 5) handed each request from grpc's polling thread to a pool
    worker and back, several GIL round trips per call: ~2.5 k calls/s on 8 cores, so 64
    closed-loop agents queued ~28 ms per upload.  On the event loop a
    SendFrame is parse (upb, C) + RRLC view (numpy, zero-copy) + a non-blocking queue put,
    ~2x the calls/s, and ClientPoll long-polls are coroutines parked on an event the model
    store sets (no thread per parked poll).  A TorchScript archive that still has to be built
    is built on a worker thread, never on the loop."""

    def __init__(self, service, address: str, idle_timeout_ms: int = 30, max_workers: int = 4,
                 max_message_mb: int = 256):
        import asyncio

        self.service = service
        self.idle_timeout_s = max(0, int(idle_timeout_ms)) / 1000.0
        self._opts = [("grpc.max_receive_message_length", max_message_mb << 20),
                      ("grpc.max_send_message_length", max_message_mb << 20)]
        addr = address.replace("tcp://", "")
        if addr.startswith("*:"):
            addr = "0.0.0.0:" + addr[2:]
        self._addr = addr
        self.bad_frames = 0
        self.rejected = 0  # uploads refused because the learner queue was full (backpressure)
        self.calls = 0
        self._pool = futures.ThreadPoolExecutor(max_workers=max(1, max_workers), thread_name_prefix="rrl-grpc-ts")
        self._loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self._err: Optional[BaseException] = None
        self._model_ev = None  # asyncio.Event, replaced after each set (created on the loop)
        self.port = 0
        self._thread = threading.Thread(target=self._run, name="rrl-grpc-aio", daemon=True)
        self._thread.start()
        self._ready.wait(30)
        if self._err is not None:
            raise self._err
        if self.port == 0:
            raise RuntimeError(f"gRPC server could not bind {address}")
        service.store.subscribe(self._on_model)

    # ------------------------------------------------------------------ loop thread
    def _run(self):
        import asyncio

        asyncio.set_event_loop(self._loop)
        try:
            self._loop.run_until_complete(self._start())
        except BaseException as e:  # noqa: BLE001 -- surfaced by __init__
            self._err = e
            self._ready.set()
            return
        self._ready.set()
        self._loop.run_forever()

    async def _start(self):
        import asyncio

        import grpc

        self._model_ev = asyncio.Event()
        self.server = grpc.aio.server(options=self._opts)
        handlers = {
            "SendActions": grpc.unary_unary_rpc_method_handler(
                self._send_actions, request_deserializer=PbTrajectory.FromString,
                response_serializer=PbResponse.SerializeToString),
            "SendFrame": grpc.unary_unary_rpc_method_handler(
                self._send_frame, request_deserializer=PbFrame.FromString,
                response_serializer=PbResponse.SerializeToString),
            "ClientPoll": grpc.unary_unary_rpc_method_handler(
                self._client_poll, request_deserializer=PbRequest.FromString,
                response_serializer=PbModel.SerializeToString),
        }
        self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
        self.port = self.server.add_insecure_port(self._addr)
        if self.port:
            await self.server.start()

    def _on_model(self, blob):
        """ModelStore subscriber (publisher's thread): wake the parked polls, O(1)."""
        if not self._loop.is_closed():
            try:
                self._loop.call_soon_threadsafe(self._wake_polls)
            except RuntimeError:  # loop stopped during shutdown
                pass

    def _wake_polls(self):
        import asyncio

        ev, self._model_ev = self._model_ev, asyncio.Event()
        ev.set()

    async def _submit(self, traj, timeout_s: float = 30.0) -> bool:
        """Queue an upload for the learner.  A full queue parks THIS call (backpressure on its
        agent, as the blocking put of the thread-pool server did) without stalling the loop."""
        import asyncio

        if self.service.submit(traj, block=False):
            return True
        deadline = self._loop.time() + timeout_s
        delay = 0.0005
        while self._loop.time() < deadline:
            await asyncio.sleep(delay)
            if self.service.submit(traj, block=False):
                return True
            delay = min(delay * 2, 0.02)
        self.rejected += 1
        return False

    # ------------------------------------------------------------------ handlers (on the loop)
    async def _send_actions(self, req, ctx):
        self.calls += 1
        try:
            traj = trajectory_from_pb(req)
            traj.agent_id = ""
            if not await self._submit(traj):
                return PbResponse(code=0, message="learner queue full: retry later")
            return PbResponse(code=1, message=f"received {len(req.actions)} actions")
        except Exception as e:  # noqa: BLE001
            return PbResponse(code=0, message=f"error: {e!r}")

    async def _send_frame(self, req, ctx):
        from ..types import TrajectoryColumns

        self.calls += 1
        try:
            f = req.frame
            traj = TrajectoryColumns.decode(f) if TrajectoryColumns.is_frame(f) else RelayRLTrajectory.decode(f)
        except Exception as e:  # noqa: BLE001
            self.bad_frames += 1
            return PbResponse(code=0, message=f"bad frame: {e!r}")
        if not await self._submit(traj):
            return PbResponse(code=0, message="learner queue full: retry later")
        return PbResponse(code=1, message=f"received {len(traj)} actions")

    async def _client_poll(self, req, ctx):
        import asyncio

        self.calls += 1
        rrlm = bool(req.first_time & 2)
        first = bool(req.first_time & 1)
        st = self.service.store
        blob = st.latest()
        if blob is None:
            return PbModel(code=-1, error="no model available")
        if not first and blob.version <= req.version:
            deadline = self._loop.time() + self.idle_timeout_s
            while True:  # parked until the store publishes a newer version or the idle timeout
                ev = self._model_ev
                blob = st.latest()
                if blob is not None and blob.version > req.version:
                    break
                left = deadline - self._loop.time()
                if left <= 0:
                    return PbModel(code=0, version=req.version)
                try:
                    await asyncio.wait_for(ev.wait(), left)
                except asyncio.TimeoutError:
                    pass
        if rrlm:
            payload = blob.encode()
        elif blob._ts is not None:
            payload = blob._ts
        else:  # an export: off the loop
            payload = await self._loop.run_in_executor(self._pool, blob.torchscript)
        return PbModel(code=1, model=payload, version=blob.version)

    def close(self, grace: float = 0.5):
        import asyncio

        self.service.store.unsubscribe(self._on_model)
        if self._loop.is_running():
            fut = asyncio.run_coroutine_threadsafe(self.server.stop(grace), self._loop)
            try:
                fut.result(timeout=10)
            except Exception:  # noqa: BLE001 -- shutting down anyway
                pass
            self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(timeout=10)
        self._pool.shutdown(wait=False)
        if not self._loop.is_running():
            self._loop.close()


# ---------------------------------------------------------------------- client
class GrpcAgentTransport:
    def __init__(self, address: str, on_model: Callable[[ModelBlob], None], connect_retries: int = 60,
                 retry_interval_s: float = 0.5, handshake_timeout_s: float = 60.0, background_poll: bool = True):
        import grpc

        self.on_model = on_model
        addr = address.replace("tcp://", "")
        if addr.startswith("*:"):
            addr = "127.0.0.1:" + addr[2:]
        self.channel = grpc.insecure_channel(addr, options=[("grpc.max_receive_message_length", 256 << 20),
                                                             ("grpc.max_send_message_length", 256 << 20)])
        last = None
        for _ in range(max(1, connect_retries)):
            try:
                grpc.channel_ready_future(self.channel).result(timeout=retry_interval_s * 4)
                last = None
                break
            except Exception as e:  # retry with a bounded budget (fixes A4)
                last = e
                time.sleep(retry_interval_s)
        if last is not None:
            raise ConnectionError(f"gRPC server {addr} unreachable: {last!r}")
        self._send = self.channel.unary_unary(f"/{SERVICE}/SendActions", request_serializer=PbTrajectory.SerializeToString,
                                              response_deserializer=PbResponse.FromString)
        self._poll = self.channel.unary_unary(f"/{SERVICE}/ClientPoll", request_serializer=PbRequest.SerializeToString,
                                              response_deserializer=PbModel.FromString)
        self.version = -1
        t0 = time.time()
        while True:  # initial handshake (agent_grpc.rs:318-360), bounded
            r = self._poll(PbRequest(first_time=3, version=-1), timeout=10)
            if r.code == 1:
                self._apply(r)
                break
            if time.time() - t0 > handshake_timeout_s:
                raise TimeoutError("gRPC model handshake timed out")
            time.sleep(retry_interval_s)
        self._sendf = self.channel.unary_unary(f"/{SERVICE}/SendFrame", request_serializer=PbFrame.SerializeToString,
                                               response_deserializer=PbResponse.FromString)
        self._stop = threading.Event()
        self._poller = None
        if background_poll:
            self._poller = threading.Thread(target=self._poll_loop, daemon=True, name="rrl-grpc-poll")
            self._poller.start()

    def _poll_loop(self):
        """Long-poll for newer models; the server parks each call up to its idle timeout."""
        while not self._stop.is_set():
            if not self.poll(timeout_s=5.0, quiet=True):
                self._stop.wait(0.005)

    def _apply(self, r):
        blob = ModelBlob.decode(r.model)
        self.version = blob.version
        self.on_model(blob)

    def send_trajectory_pb(self, traj: RelayRLTrajectory) -> bool:
        from ..utils.faults import injector

        inj = injector()
        if inj.enabled and inj.filter_upload(b"x" * 32) is None:
            return True  # injected loss
        try:
            r = self._send(trajectory_to_pb(traj), timeout=30)
            return r.code == 1
        except Exception as e:
            print(f"[GrpcAgentTransport] SendActions failed: {e!r}", flush=True)
            return False

    def send_frame(self, frame: bytes) -> bool:
        from ..utils.faults import injector

        frame = injector().filter_upload(frame)
        if frame is None:
            return True  # injected loss
        try:
            return self._sendf(PbFrame(frame=frame), timeout=30).code == 1
        except Exception as e:
            print(f"[GrpcAgentTransport] SendFrame failed: {e!r}", flush=True)
            return False

    def poll(self, timeout_s: float = 5.0, quiet: bool = False) -> bool:
        try:
            r = self._poll(PbRequest(first_time=2, version=self.version), timeout=timeout_s)
        except Exception as e:
            if not quiet and not self._stop.is_set():
                print(f"[GrpcAgentTransport] ClientPoll failed: {e!r}", flush=True)
            if quiet:
                self._stop.wait(0.2)
            return False
        if r.code == 1 and r.version > self.version:
            self._apply(r)
            return True
        return False

    def close(self):
        self._stop.set()
        if self._poller is not None:
            self._poller.join(timeout=6)
        self.channel.close()


class ReferenceGrpcAgentTransport:
    """The reference gRPC agent's wire (agent_grpc.rs:318-360 handshake, 492-533 SendActions,
    540-599 poll and swap; grpc_utils.rs:31-129 action codec, 196-205 model decode).

    Differences by design: the archive is read from its raw zip storages
    (``utils.checkpoint.reference_weights_from_bytes``, nothing unpickled, no tempfile); an RPC
    error is reported instead of ``process::exit(1)`` (agent_grpc.rs:528-531); the handshake
    is bounded by ``handshake_timeout_s``.  The reference server always answers version 0
    (training_grpc.rs:724,746,775), so ``server_version`` is echoed back as the reference does
    and ``version`` counts the models this agent actually loaded."""

    def __init__(self, address: str, on_model: Callable[[ModelBlob], None], handshake_timeout_s: float = 60.0,
                 retry_interval_s: float = 0.5, rpc_timeout_s: float = 30.0):
        import grpc

        self.on_model = on_model
        self.rpc_timeout_s = rpc_timeout_s
        addr = address.replace("tcp://", "")
        if addr.startswith("*:"):
            addr = "127.0.0.1:" + addr[2:]
        self.channel = grpc.insecure_channel(addr, options=[("grpc.max_receive_message_length", 256 << 20),
                                                             ("grpc.max_send_message_length", 256 << 20)])
        self._send = self.channel.unary_unary(f"/{SERVICE}/SendActions", request_serializer=PbTrajectory.SerializeToString,
                                              response_deserializer=PbResponse.FromString)
        self._poll = self.channel.unary_unary(f"/{SERVICE}/ClientPoll", request_serializer=PbRequest.SerializeToString,
                                              response_deserializer=PbModel.FromString)
        self.version = 0          # models loaded by this agent
        self.server_version = 0   # the version field the server last answered (echoed in polls)
        self.bad_models = 0
        self.rejected = 0
        t0 = time.time()
        while True:
            try:
                r = self._poll(PbRequest(first_time=1, version=0), timeout=10)
                if r.code == 1 and len(r.model) and self._load(r):
                    break
            except Exception as e:  # noqa: BLE001 -- server not up yet: retry like the reference
                if time.time() - t0 > handshake_timeout_s:
                    raise ConnectionError(f"gRPC server {addr}: {e!r}")
            if time.time() - t0 > handshake_timeout_s:
                raise TimeoutError("reference gRPC model handshake timed out")
            time.sleep(retry_interval_s)  # agent_grpc.rs:357 (500 ms)

    def _load(self, r) -> bool:
        from ..runtime.model_store import blob_from_archive

        try:
            self.on_model(blob_from_archive(self.version + 1, bytes(r.model)))
        except Exception as e:  # noqa: BLE001 -- a model the agent cannot validate is skipped
            self.bad_models += 1
            print(f"[ReferenceGrpcAgentTransport] bad model: {e!r}", flush=True)
            return False
        self.version += 1
        self.server_version = int(r.version)
        return True

    def send_actions(self, actions) -> bool:
        """One episode (its actions + the terminal marker) as ``SendActions``; on acceptance one
        ``ClientPoll{first_time: 0}`` that swaps in a newer model if the server has one."""
        from ..utils.faults import injector

        inj = injector()
        if inj.enabled and inj.filter_upload(b"x" * 32) is None:
            return True  # injected loss
        msg = PbTrajectory(actions=[action_to_pb(a) for a in actions])
        for m in msg.actions:
            m.reward_update_flag = False  # grpc_utils.rs:64 hard-codes it
        try:
            r = self._send(msg, timeout=self.rpc_timeout_s)
        except Exception as e:  # noqa: BLE001 -- reported, not process::exit(1)
            print(f"[ReferenceGrpcAgentTransport] SendActions failed: {e!r}", flush=True)
            return False
        if r.code != 1:
            self.rejected += 1
            return False
        self.poll()
        return True

    def poll(self) -> bool:
        try:
            r = self._poll(PbRequest(first_time=0, version=self.server_version), timeout=self.rpc_timeout_s)
        except Exception as e:  # noqa: BLE001
            print(f"[ReferenceGrpcAgentTransport] ClientPoll failed: {e!r}", flush=True)
            return False
        if r.code == 1 and len(r.model):
            return self._load(r)
        return False

    def heartbeat(self):
        pass

    def close(self):
        self.channel.close()
