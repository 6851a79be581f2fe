"""EngineRunner's threshold check one epoch behind (log_every=0): epoch k's episode sums are
read after epoch k + 1 is queued, so the device stream never drains for the check.  Same
window means as the synchronous check, solved one epoch later, the last epoch's sums
consumed when the loop ends for another reason."""
import pytest

from relayrl_prototype_amd.runtime.engine import EngineRunner
from relayrl_prototype_amd.runtime.vec_trainer import PendingSums


class _Trainer:
    env_steps = 0


class _Service:
    updates = 0

    def publish_model(self):
        pass


class _Algo:
    publishes_policy = False
    comm = None

    def __init__(self, per_epoch, async_trainer=True):
        self.per_epoch = per_epoch  # (episodes, return sum) of each epoch
        self.epoch = 0
        self.trainer = _Trainer()
        if async_trainer:  # like VecTrainer: a non-draining read exists
            self.trainer.episode_sums_async = self.episode_sums_async
        self.reads = []  # epochs whose sums were read, in order, and when (epochs done then)

    def train_model(self):
        self.epoch += 1

    def epoch_metrics(self):
        return {}

    def episode_sums(self, m=None):
        self.reads.append((self.epoch, self.epoch))
        return self.per_epoch[self.epoch - 1]

    def episode_sums_async(self):
        k = self.epoch
        algo = self

        class _H(PendingSums):
            def result(self):
                algo.reads.append((k, algo.epoch))
                return algo.per_epoch[k - 1]
        return _H(None)

    def log_epoch(self, m, extra=None):
        pass


SUMS = [(10, 100.0), (10, 300.0), (10, 480.0), (10, 490.0), (10, 500.0), (10, 500.0)]


@pytest.mark.parametrize("lagged", ["1", "0"])
def test_lagged_check_solves_one_epoch_later(lagged, monkeypatch):
    monkeypatch.setenv("RRL_TTT_LAGGED_CHECK", lagged)
    algo = _Algo(SUMS)
    r = EngineRunner(algo, _Service(), 0.0).train(epochs=10, target_return=47.5, window=10, log_every=0)
    assert r.solved and r.last_window_return == pytest.approx(48.0)
    if lagged == "1":
        # epoch 3 (the first solved) is read while epoch 4 has already run
        assert algo.reads == [(1, 2), (2, 3), (3, 4)] and r.epochs == 4
    else:
        assert algo.reads == [(1, 1), (2, 2), (3, 3)] and r.epochs == 3


def test_lagged_check_reads_the_last_epoch_at_the_end(monkeypatch):
    monkeypatch.setenv("RRL_TTT_LAGGED_CHECK", "1")
    algo = _Algo(SUMS)
    r = EngineRunner(algo, _Service(), 0.0).train(epochs=3, target_return=47.5, window=10, log_every=0)
    # the loop stops at the epoch limit with epoch 3's sums unread; they are read after it
    assert algo.reads == [(1, 2), (2, 3), (3, 3)]
    assert r.epochs == 3 and r.solved and r.last_window_return == pytest.approx(48.0)


def test_logging_keeps_the_synchronous_check(monkeypatch):
    monkeypatch.setenv("RRL_TTT_LAGGED_CHECK", "1")
    algo = _Algo(SUMS)
    r = EngineRunner(algo, _Service(), 0.0).train(epochs=10, target_return=47.5, window=10, log_every=1)
    assert r.epochs == 3 and [k for k, _ in algo.reads] == [1, 2, 3]


def test_trainers_without_an_async_read_keep_the_synchronous_check(monkeypatch):
    """host / pixel / actor-learner trainers have no non-draining read; the lag
    would only add an epoch past the threshold (TTT, epoch count and final model off by one)."""
    monkeypatch.setenv("RRL_TTT_LAGGED_CHECK", "1")
    algo = _Algo(SUMS, async_trainer=False)
    r = EngineRunner(algo, _Service(), 0.0).train(epochs=10, target_return=47.5, window=10, log_every=0)
    assert r.epochs == 3 and algo.reads == [(1, 1), (2, 2), (3, 3)]
