"""World-size-2 `gloo` test of the multi-GPU sharding + gather path (CPU).

Each rank computes its shard of independent pairs (here with the oracle: the CPU suite
has no GPU) and rank 0 gathers the disparity maps; the gathered batch must be
byte-identical to a single-process run over all pairs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tea_stereo_matching_amd import distributed as D
from tea_stereo_matching_amd import synthetic as S

H, W, L, B = 24, 40, 9, 2  # tiny pairs, 2 per rank


def _compute(idx):
    from oracle import oracle as O

    left, right, _ = S.make_scene(D.pair_seed(idx), H, W, L)
    d, _ = O.compute(left, right, O.default_params(O.RGB, 0, L - 1, num_threads=1))
    return d


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = torch.from_numpy(np.stack([_compute(i) for i in D.shard(rank, B)]))
        got = D.gather_to_root(mine, rank, world)
        t = D.max_over_ranks(float(rank + 1), world)
        if rank == 0:
            np.save(out_path, torch.cat(got).numpy())
            assert t == float(world)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_is_a_partition():
    seen = [i for r in range(4) for i in D.shard(r, 3)]
    assert seen == list(range(12))
    assert D.pair_seed(0) == 1000


def test_gloo_world2_gather_matches_single_process(tmp_path, oracle):
    out = str(tmp_path / "gathered.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    gathered = np.load(out)
    single = np.stack([_compute(i) for i in range(2 * B)])
    assert gathered.shape == (2 * B, H, W)
    assert np.array_equal(gathered, single)
