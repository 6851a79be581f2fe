"""The threshold check's device side: column_sums (scan.hip) against a float64 torch sum, and
VecTrainer.episode_sums_async() against the synchronous episode_sums() over real epochs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,ld,cols", [(1, 8, 2), (37, 8, 2), (1024, 8, 8), (5000, 3, 3)])
def test_column_sums_matches_float64(cuda, rows, ld, cols):
    from relayrl_prototype_amd.ops import hip

    g = torch.Generator().manual_seed(rows)
    x = (torch.rand(rows, ld, generator=g) * 100).to(cuda)
    out = torch.full((cols,), float("nan"), dtype=torch.float64, device=cuda)
    hip().column_sums(x, cols, out)
    torch.testing.assert_close(out.cpu(), x.double().cpu()[:, :cols].sum(0), rtol=1e-12, atol=1e-9)


def test_episode_sums_async_equals_the_synchronous_read(cuda):
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    tr = VecTrainer(VecTrainerConfig(num_envs=512, rollout_len=16, train_vf_iters=3, seed=4), device=cuda)
    pending, prev, total = None, None, 0.0
    for _ in range(6):  # the engine's pattern: epoch k's handle read after epoch k + 1's is taken
        tr.train_epoch()
        h = tr.episode_sums_async()
        n, s = tr.episode_sums()
        total += n
        if pending is not None:
            hn, hs = pending.result()
            assert hn == prev[0] and hs == pytest.approx(prev[1], rel=1e-6)
        pending, prev = h, (n, s)
    hn, hs = pending.result()
    assert hn == prev[0] and hs == pytest.approx(prev[1], rel=1e-6)
    assert total > 0
