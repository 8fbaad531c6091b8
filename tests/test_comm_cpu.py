"""Control-plane agreement of the p2p transport (parallel/comm.py agree): a pre-flight that
fails on ONE rank must switch every rank to the fallback -- with an explicit group and with
group=None (the world group the schedule API passes)."""
import pytest

from dist_utils import run_world


def _vote(rank, world, use_world):
    import torch
    import torch.distributed as dist
    from mipipe.parallel.comm import agree

    group = None if use_world else dist.new_group(list(range(world)), backend="gloo")
    ok_all = agree(True, group, torch.device("cpu"))
    one_fails = agree(rank != world - 1, group, torch.device("cpu"))
    return ok_all, one_fails


@pytest.mark.parametrize("use_world", [True, False])
def test_one_failing_rank_fails_the_vote_everywhere(use_world):
    res = run_world(_vote, 3, use_world)
    for r in range(3):
        assert res[r] == (True, False), res
