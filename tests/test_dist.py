"""The N > 1 path on CPU: two gloo ranks shard a population, evaluate their
rows (the oracle stands in for the device kernel here) and all-gather the
fitness; the result must equal the single-process evaluation exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    from pong_amd.dist import shard_range
    for n in (0, 1, 7, 64, 65536, 524288 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _worker(rank, world, port, shape, genomes, opponents, kinds, opp, mult, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        repo = os.path.dirname(here)
        sys.path.insert(0, os.path.join(repo, "oracle"))
        sys.path.insert(0, os.path.join(repo, "neuro-genetic-pong-self-play_amd"))
        import oracle as O
        from pong_amd.dist import evaluate_sharded

        def rows(lo, hi):
            r = O.eval_population(genomes[lo:hi], shape, kinds[lo:hi], opp[lo:hi], mult[lo:hi],
                                  opponents=opponents)
            return torch.from_numpy(r["fitness"])

        full = evaluate_sharded(rows, genomes.shape[0])
        if rank == 0:
            np.save(out_path, full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [37, 64])
def test_two_rank_sharded_evaluation(oracle, tmp_path, n):
    shape = [6, 2, 2]
    rng = np.random.default_rng(n)
    genomes = rng.standard_normal((n, 20)) * 3
    opponents = rng.standard_normal((5, 20)) * 3
    kinds = np.tile(np.array([0, 1, 2, 3, 3, 3], np.int32), (n, 1))
    opp = rng.integers(0, 5, size=(n, 6)).astype(np.int32)
    mult = np.where(kinds == 3, rng.normal(size=(n, 6)), 1.0)
    out = tmp_path / "fit.npy"
    mp.spawn(_worker, args=(2, _free_port(), shape, genomes, opponents, kinds, opp, mult, str(out)),
             nprocs=2, join=True)
    single = oracle.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents)["fitness"]
    np.testing.assert_array_equal(np.load(out), single)


def test_deal_positions_snake_partition():
    """The length-balanced shards' deal (DeviceGA.balance_shards): the ranks'
    positions partition [0, N * n), each rank's k-th position lies in round k,
    and a descending list dealt this way leaves the ranks' sums within one
    element of each other."""
    from pong_amd.dist import deal_positions
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        n = 13
        pos = [deal_positions(n, r, world).numpy() for r in range(world)]
        allp = np.sort(np.concatenate(pos))
        np.testing.assert_array_equal(allp, np.arange(world * n))
        for p in pos:
            np.testing.assert_array_equal(p // world, np.arange(n))
        lengths = np.sort(rng.integers(1, 2000, size=world * n))[::-1]
        sums = [lengths[p].sum() for p in pos]
        assert max(sums) - min(sums) <= lengths[0]


def _gather_equal_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.join(os.path.dirname(here), "neuro-genetic-pong-self-play_amd"))
        from pong_amd.dist import gather_equal
        local = torch.tensor([[rank, 10.0 * rank + k] for k in range(3)], dtype=torch.float64)
        out = gather_equal(local)
        if rank == 0:
            np.save(out_path, out.numpy())
    finally:
        dist.destroy_process_group()


def test_gather_equal_two_ranks(tmp_path):
    out = str(tmp_path / "g.npy")
    mp.spawn(_gather_equal_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    np.testing.assert_array_equal(got, np.array([[0, 0], [0, 1], [0, 2], [1, 10], [1, 11], [1, 12]], np.float64))
