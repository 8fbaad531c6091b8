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


def _dp_transport(rank, world, wanted_by):
    """pp=2 x dp=2: ranks in ``wanted_by`` see a native pipeline engine (the others'
    pre-flight fell back).  The DP engine must be built on all ranks or on none."""
    import torch
    from mipipe.parallel import collectives as C
    from mipipe.parallel.mesh import build_mesh
    mesh = build_mesh(2, 2, torch.device("cpu"))
    built = []
    C.Collectives._dp_native_wanted = lambda self: rank in wanted_by
    C.make_dp_engine = lambda *a, **k: built.append(1) or object()
    coll = C.Collectives(mesh, torch.device("cpu"))
    return coll.dp_kind, len(built)


@pytest.mark.parametrize("wanted_by", [(0, 1), (0, 1, 2, 3)])
def test_dp_transport_is_agreed_over_the_world(wanted_by):
    """one DP replica's pipeline falling back to torch p2p must not leave the
    other replica entering the native DP engine's broadcast + communicator init alone."""
    res = run_world(_dp_transport, 4, wanted_by)
    kinds = {res[r] for r in range(4)}
    assert len(kinds) == 1, res
    assert kinds == ({("native", 1)} if len(wanted_by) == 4 else {("torch", 0)}), res
