"""The native gRPC server (csrc/net/h2grpc.cpp, HTTP/2 via nghttp2, one epoll thread): the
RelayRLRoute RPCs answered in C++ against a stock grpcio client -- uploads queued without the
GIL, parked long polls, TorchScript on demand, backpressure, unknown methods -- and the
TrainingServer using it by default (gRPC fan-in under the GIL)."""
import concurrent.futures as cf
import threading
import time

import grpc
import pytest

from relayrl_prototype_amd.transport.grpc_transport import (SERVICE, PbAction, PbFrame, PbModel, PbRequest,
                                                             PbResponse, PbTrajectory)
from relayrl_prototype_amd.transport.h2_native import load

from test_api_e2e import cfgdir, run_episodes  # noqa: F401

mod = load()
pytestmark = pytest.mark.skipif(mod is None, reason="native gRPC module not built (nghttp2 missing)")


def _stubs(port):
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    mk = lambda name, req, rsp: ch.unary_unary(f"/{SERVICE}/{name}", request_serializer=req.SerializeToString,  # noqa: E731
                                               response_deserializer=rsp.FromString)
    return ch, mk("SendFrame", PbFrame, PbResponse), mk("ClientPoll", PbRequest, PbModel), \
        mk("SendActions", PbTrajectory, PbResponse)


def test_rpcs_long_poll_and_torchscript_on_demand():
    s = mod.GrpcServer("127.0.0.1", 0, idle_timeout_ms=300)
    ch, send, poll, acts = _stubs(s.port)
    try:
        r = poll(PbRequest(first_time=3, version=-1), timeout=5)
        assert r.code == -1 and r.error == "no model available"
        s.set_model(1, b"RRLM-one", None)
        assert send(PbFrame(frame=b"episode" * 500), timeout=5).code == 1
        kind, body, _ = s.recv(1000)
        assert kind == mod.FRAME and body == b"episode" * 500
        r = poll(PbRequest(first_time=3, version=-1), timeout=5)
        assert (r.code, r.model, r.version) == (1, b"RRLM-one", 1)
        t0 = time.time()
        r = poll(PbRequest(first_time=2, version=1), timeout=5)  # nothing newer: the idle timeout
        assert r.code == 0 and r.version == 1 and 0.25 < time.time() - t0 < 2.0
        threading.Timer(0.1, lambda: s.set_model(2, b"RRLM-two", None)).start()
        t0 = time.time()
        r = poll(PbRequest(first_time=2, version=1), timeout=5)  # parked, answered by the publish
        assert (r.code, r.model, r.version) == (1, b"RRLM-two", 2) and time.time() - t0 < 0.3

        def build_ts():  # the consumer side: a reference-dialect poll asks for the archive once
            kind, _, ver = s.recv(2000)
            assert kind == mod.NEED_TS and ver == 2
            s.set_model_ts(ver, b"TS-two")

        th = threading.Thread(target=build_ts)
        th.start()
        r = poll(PbRequest(first_time=1, version=0), timeout=5)
        th.join()
        assert (r.code, r.model, r.version) == (1, b"TS-two", 2)
        assert acts(PbTrajectory(actions=[PbAction(reward=1.0, done=True)]), timeout=5).code == 1
        kind, body, _ = s.recv(1000)
        assert kind == mod.ACTIONS and PbTrajectory.FromString(body).actions[0].done
        big = b"x" * (3 << 20)
        assert send(PbFrame(frame=big), timeout=10).code == 1 and s.recv(1000)[1] == big
        with pytest.raises(grpc.RpcError) as ei:
            ch.unary_unary(f"/{SERVICE}/Nope", request_serializer=PbFrame.SerializeToString)(PbFrame(), timeout=5)
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
    finally:
        ch.close()
        s.close()


def test_concurrent_uploads_and_backpressure_in_order():
    s = mod.GrpcServer("127.0.0.1", 0, max_inbox=4)
    ch, send, _, _ = _stubs(s.port)
    try:
        done = []

        def one(i):
            r = send(PbFrame(frame=b"%06d" % i), timeout=20)
            done.append(i)
            return r.code

        with cf.ThreadPoolExecutor(16) as ex:
            futs = [ex.submit(one, i) for i in range(64)]
            time.sleep(0.5)
            assert len(done) <= 8  # only what fits the 4-item inbox was answered; the rest is parked
            got = []
            while len(got) < 64:
                it = s.recv(5000)
                assert it is not None
                got.append(int(it[1]))
            assert all(f.result() == 1 for f in futs)
        assert sorted(got) == list(range(64)) and s.stats()["inbox_waits"] > 0
    finally:
        ch.close()
        s.close()


def test_training_server_uses_the_native_server(cfgdir):  # noqa: F811
    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.api.server import TrainingServer
    from relayrl_prototype_amd.transport.grpc_transport import NativeGrpcTrainingEndpoint

    tmp, cfgp = cfgdir
    srv = TrainingServer("REINFORCE", 4, 2, 100000, env_dir=str(tmp / "env"), config_path=cfgp, server_type="grpc",
                         device="cpu")
    try:
        ep = srv._endpoints[0]
        assert isinstance(ep, NativeGrpcTrainingEndpoint)
        for wire in ("columns", "actions", "reference"):
            agent = RelayRLAgent(config_path=cfgp, server_type="grpc", handshake_timeout_s=30, wire_format=wire)
            run_episodes(agent, 4, max_steps=50)
            agent.close()
        t0 = time.time()
        while srv.service.received < 12 and time.time() - t0 < 20:
            time.sleep(0.02)
        assert srv.service.received == 12 and srv.service.errors == 0 and ep.bad_frames == 0
        st = ep.stats()
        assert st["frames"] >= 4 and st["actions"] >= 8 and st["polls"] >= 3
    finally:
        srv.close(save=False)


def test_oversized_requests_are_refused_and_the_server_lives():
    """max_request caps one message and twice that caps what one connection may hold (bodies in
    flight + uploads parked on a full inbox): larger uploads are refused with a stream reset
    instead of being buffered, and the connection keeps serving."""
    s = mod.GrpcServer("127.0.0.1", 0, max_inbox=1, max_request=256 << 10)
    ch, send, _, _ = _stubs(s.port)
    try:
        with pytest.raises(grpc.RpcError):
            send(PbFrame(frame=b"y" * (300 << 10)), timeout=10)
        assert send(PbFrame(frame=b"small"), timeout=10).code == 1
        assert s.recv(1000)[1] == b"small"
        # the inbox holds one item: park uploads of 200 KB until the connection's 2 x 256 KB is
        # reached -- the rest are refused, nothing is buffered past the cap
        assert send(PbFrame(frame=b"first"), timeout=10).code == 1  # fills the 1-item inbox
        with cf.ThreadPoolExecutor(8) as ex:
            futs = [ex.submit(send, PbFrame(frame=bytes([i]) * (200 << 10)), timeout=20) for i in range(8)]
            time.sleep(1.0)
            got = [s.recv(2000) for _ in range(9)]
            ok = err = 0
            for f in futs:
                try:
                    ok += f.result().code == 1
                except grpc.RpcError:
                    err += 1
        assert ok >= 2 and err >= 1 and ok + err == 8, (ok, err)
        assert got[0][1] == b"first" and sum(g is not None for g in got) == 1 + ok
        assert s.stats()["refused_streams"] >= err
        assert send(PbFrame(frame=b"after"), timeout=10).code == 1 and s.recv(1000)[1] == b"after"
    finally:
        ch.close()
        s.close()
