"""NCCL (RCCL) stream semantics of the actor-learner schedule, on the CPU.

gloo tests cannot show head-of-line blocking: gloo progresses every posted send / receive
independently.  Under NCCL every operation of a process group runs on ONE stream per rank
(``batch_isend_irecv`` on the default group uses the group's main communicator, like its
collectives), in issue order, and a send only completes while the matching receive is
running at the head of the peer's stream.  ``Work.wait()`` does not block the host: it makes
the compute stream wait for the operation, and every later NCCL launch waits for the compute
stream (ProcessGroupNCCL syncs its stream with the current stream at issue).

The real ``ActorLearner.step`` (runtime/actor_learner.py:294-402) runs here for every rank of
a W-rank job against a recording fake of ``torch.distributed`` (CPU tensors, host envs, the
oracle learner); each rank's trace -- P2P batches, collectives per process group, waits, and
the Rollout / Learn compute phases -- is then replayed by a simulator of those semantics:

* every schedule (L learner shards in {1, 2, 4}, K actor blocks per shard in {1, 2, 4},
  max_lag in {0, 1}) completes: no deadlock;
* the intended overlap holds: with a learner stalled inside its update k, an actor-only rank
  still runs rollout k + 1 at max_lag 1, and cannot at max_lag 0;
* a deliberately swapped order -- the actor posting irecv(weights) before isend(rollout) --
  deadlocks in the simulator (it passes under gloo).
"""
import itertools
from collections import defaultdict, deque

import pytest
import torch

from relayrl_prototype_amd.parallel import comm as comm_mod
from relayrl_prototype_amd.parallel.comm import Comm
from relayrl_prototype_amd.runtime import actor_learner as al_mod
from relayrl_prototype_amd.runtime.actor_learner import ActorLearner, ActorLearnerConfig


# ---------------------------------------------------------------------- recording fake dist
class _Group:
    def __init__(self, ranks):
        self.ranks = tuple(ranks)


WORLD = "world"


class _Work:
    def __init__(self, rec, op_id):
        self.rec, self.op_id = rec, op_id

    def wait(self):
        self.rec.events[self.rec.rank].append(("wait", self.op_id))
        return True

    def is_completed(self):
        return False


class _P2POp:
    def __init__(self, op, tensor, peer, group=None, tag=0):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group


class FakeDist:
    """The subset of torch.distributed that comm.py and actor_learner.py call, recording."""

    P2POp = _P2POp

    class ReduceOp:
        SUM, MAX, MIN = "sum", "max", "min"

    def __init__(self, world):
        self.world = world
        self.rank = 0
        self.events = defaultdict(list)
        self.ops = {}  # op id -> dict

    # ops (distinct sentinels: P2POp records which one it was given)
    @staticmethod
    def isend(*a, **k):
        raise AssertionError("point-to-point ops go through batch_isend_irecv")

    @staticmethod
    def irecv(*a, **k):
        raise AssertionError("point-to-point ops go through batch_isend_irecv")

    def _pg(self, group):
        return WORLD if group is None else group.ranks

    def _issue(self, **op):
        oid = len(self.ops)
        op.update(rank=self.rank, id=oid)
        self.ops[oid] = op
        self.events[self.rank].append(("issue", oid))
        return oid

    def batch_isend_irecv(self, ops):
        items = [("send" if o.op is FakeDist.isend else "recv", int(o.peer)) for o in ops]
        oid = self._issue(kind="p2p", pg=self._pg(ops[0].group), items=items)
        return [_Work(self, oid) for _ in ops]

    def _coll(self, name, group, async_op):
        oid = self._issue(kind="coll", pg=self._pg(group), name=name)
        w = _Work(self, oid)
        if async_op:
            return w
        w.wait()  # a synchronous NCCL collective = the current stream waits for it
        return None

    def all_reduce(self, t, op=None, group=None, async_op=False):
        return self._coll("all_reduce", group, async_op)

    def broadcast(self, t, src=0, group=None, async_op=False):
        return self._coll("broadcast", group, async_op)

    def barrier(self, group=None, **kw):
        return self._coll("barrier", group, False)

    def new_group(self, ranks, timeout=None, **kw):
        return _Group(ranks)

    # queries
    def is_available(self):
        return True

    def is_initialized(self):
        return True

    def get_world_size(self, group=None):
        return self.world if group is None else len(group.ranks)

    def get_rank(self, group=None):
        return self.rank if group is None else group.ranks.index(self.rank)

    def get_backend(self, group=None):
        return "nccl"


class RecTimer:
    """PhaseTimer stand-in: the Rollout / Learn phases become compute events of the trace."""

    enabled = False  # Comm.all_reduce_sum_ takes its plain path

    def __init__(self, fd, step_of):
        self.fd, self.step_of = fd, step_of

    def phase(self, name):
        import contextlib

        if name in ("Rollout", "Learn"):
            self.fd.events[self.fd.rank].append(("compute", (name, self.step_of())))
        return contextlib.nullcontext()

    def columns(self):
        return {}

    def reset(self):
        pass


# ---------------------------------------------------------------------- NCCL stream simulator
def simulate(fd: FakeDist, stalled=frozenset()):
    """Replay the traces.  ``stalled``: {(rank, (phase, step))} compute events that never
    finish.  Returns (done op ids, {rank: finished compute labels}, stuck op ids)."""
    ranks = sorted(fd.events)
    # per rank: compute-stream entries and, per issued op, how much of that stream precedes it
    cstream = {r: [] for r in ranks}
    queues = defaultdict(deque)  # (rank, pg) -> op ids in issue order
    need = {}
    for r in ranks:
        for ev in fd.events[r]:
            if ev[0] == "issue":
                op = fd.ops[ev[1]]
                need[op["id"]] = len(cstream[r])
                queues[(r, op["pg"])].append(op["id"])
            else:
                cstream[r].append(ev)
    pos = {r: 0 for r in ranks}
    done = set()
    finished = defaultdict(list)
    matched = {oid: [False] * len(op["items"]) for oid, op in fd.ops.items() if op["kind"] == "p2p"}
    coll_seq = {}
    seq_ctr = defaultdict(int)
    for r in ranks:
        for ev in fd.events[r]:
            if ev[0] == "issue" and fd.ops[ev[1]]["kind"] == "coll":
                op = fd.ops[ev[1]]
                coll_seq[op["id"]] = seq_ctr[(r, op["pg"])]
                seq_ctr[(r, op["pg"])] += 1

    def members(pg):
        return ranks if pg == WORLD else list(pg)

    def active_head(r, pg):
        q = queues[(r, pg)]
        if not q:
            return None
        oid = q[0]
        return oid if need[oid] <= pos[r] else None

    progress = True
    while progress:
        progress = False
        for r in ranks:  # compute streams
            while pos[r] < len(cstream[r]):
                ev = cstream[r][pos[r]]
                if ev[0] == "wait" and ev[1] not in done:
                    break
                if ev[0] == "compute":
                    if (r, ev[1]) in stalled:
                        break
                    finished[r].append(ev[1])
                pos[r] += 1
                progress = True
        for (r, pg) in list(queues):
            oid = active_head(r, pg)
            if oid is None:
                continue
            op = fd.ops[oid]
            if op["kind"] == "coll":
                heads = [active_head(m, pg) for m in members(pg)]
                if all(h is not None and fd.ops[h]["kind"] == "coll" and coll_seq[h] == coll_seq[oid]
                       for h in heads):
                    for m, h in zip(members(pg), heads):
                        done.add(h)
                        queues[(m, pg)].popleft()
                    progress = True
                continue
            for i, (kind, peer) in enumerate(op["items"]):
                if matched[oid][i] or kind != "send":
                    continue
                h = active_head(peer, pg)
                if h is None or fd.ops[h]["kind"] != "p2p":
                    continue
                for jj, (k2, p2) in enumerate(fd.ops[h]["items"]):
                    if k2 == "recv" and p2 == r and not matched[h][jj]:
                        matched[oid][i] = matched[h][jj] = True  # first unmatched: per-pair FIFO
                        progress = True
                        break
        for (r, pg), q in queues.items():
            while q and fd.ops[q[0]]["kind"] == "p2p" and all(matched[q[0]]):
                done.add(q.popleft())
                progress = True
    stuck = [oid for oid in fd.ops if oid not in done]
    return done, finished, stuck


# ---------------------------------------------------------------------- driver
def run_schedule(monkeypatch, L, K, max_lag, steps=4, swap=False):
    """Build every rank's ActorLearner against the recording dist and run ``steps`` steps."""
    learner_acts = True
    W = L * K
    fd = FakeDist(W)
    monkeypatch.setattr(al_mod, "dist", fd)
    monkeypatch.setattr(comm_mod, "dist", fd)
    cfg = ActorLearnerConfig(env="CartPole-v1", num_envs=2, rollout_len=4, train_vf_iters=1, num_threads=1,
                             learner_ranks=L, learner_acts=learner_acts, max_lag=max_lag, stall_timeout_s=0.0,
                             use_graphs=False)
    ranks = []
    for r in range(W):
        fd.rank = r
        a = ActorLearner(cfg, Comm(collectives=False), torch.device("cpu"))
        a.timer = RecTimer(fd, (lambda a=a: a.epoch))
        if a.lcomm is not None:
            a.lcomm.timer = None
        if swap and not a.is_learner:
            # the deliberately wrong order: post irecv(weights) before isend(rollout)
            def step(self=a):
                parts = self.actor.rollout(self.version_in_use)
                self.timer.phase("Rollout")
                self._recv_weights()
                self._send_rollout(parts)
                self.version += 1
                self.epoch += 1

            a.step = step
        ranks.append(a)
    for r, a in enumerate(ranks):
        fd.rank = r
        for _ in range(steps):
            a.step()
        if not swap:
            a.finish()
    return fd, ranks


CASES = [(L, K, lag) for L, K, lag in itertools.product((1, 2, 4), (1, 2, 4), (0, 1))]


@pytest.mark.parametrize("L,K,lag", CASES)
def test_schedule_completes_under_nccl_stream_semantics(monkeypatch, L, K, lag):
    fd, ranks = run_schedule(monkeypatch, L, K, lag)
    done, finished, stuck = simulate(fd)
    assert not stuck, f"deadlock: ops {[fd.ops[o] for o in stuck[:4]]}"
    for r, a in enumerate(ranks):
        assert ("Rollout", 3) in finished[r]


@pytest.mark.parametrize("L,K", [(1, 2), (2, 2), (1, 4), (2, 4), (4, 2)])
def test_lag1_overlaps_actor_rollout_with_the_update(monkeypatch, L, K):
    """A learner stalled inside update k: at max_lag 1 its actor-only ranks still run rollout
    k + 1 (IMPALA-style overlap); at max_lag 0 they cannot."""
    for lag, expect in ((1, True), (0, False)):
        fd, ranks = run_schedule(monkeypatch, L, K, lag)
        k = 1
        stalled = {(r, ("Learn", k)) for r, a in enumerate(ranks) if a.is_learner}
        _, finished, _ = simulate(fd, stalled)
        actors = [r for r, a in enumerate(ranks) if not a.is_learner]
        assert actors
        for r in actors:
            assert (("Rollout", k + 1) in finished[r]) is expect, (lag, r, finished[r])


@pytest.mark.parametrize("lag", [0, 1])
def test_swapped_irecv_isend_order_deadlocks(monkeypatch, lag):
    fd, _ = run_schedule(monkeypatch, 1, 2, lag, steps=2, swap=True)
    _, _, stuck = simulate(fd)
    assert stuck, "the simulator must catch the head-of-line deadlock"
