"""Multi-rank path on the CPU (gloo, world_size 2): batch sharding and the
one exchange step (the global mean_stddev all-reduce of SURVEY.md 8e)."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    from vacv_amd.dist import shard_range
    for total in [0, 1, 7, 8, 1024, 1025]:
        for world in [1, 2, 3, 8]:
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, images, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(repo, "oracle"), os.path.join(repo, "arm-neon-opencv_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from oracle import Oracle
    from vacv_amd.dist import allreduce_sums, allreduce_sums_async, shard_range, stats_from_moments
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard_range(len(images), rank, world)
    O = Oracle()
    # per-rank channel sums of its shard (on a GPU box: vacv_channel_sums)
    local = np.zeros((3, 2))
    for img in images[b:e]:
        local += O.channel_sums(img).reshape(3, 2)
    h, w = images[0].shape[:2]
    total, count = allreduce_sums(torch.from_numpy(local), float((e - b) * h * w))
    mean, std = stats_from_moments(total, count)
    # the no-sync variant bench.py's cubic_stats step uses: identical results
    ta, ca = allreduce_sums_async(torch.from_numpy(local), float((e - b) * h * w))
    ma, sa = stats_from_moments(ta, ca)
    assert float(ca) == count and torch.equal(ma, mean) and torch.equal(sa, std)
    out_q.put((rank, mean.numpy(), std.numpy(), count))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_images", [5, 8])
def test_global_stats_allreduce_gloo(n_images):
    from oracle import Oracle, synthetic_image
    images = [synthetic_image(500 + k, 48, 64, 3) for k in range(n_images)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, images, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    O = Oracle()
    full = np.concatenate([im.reshape(-1, 3) for im in images])[None]
    want_m, want_s = O.mean_stddev_exact(full)
    for rank, m, s, count in res:
        assert count == n_images * 48 * 64
        assert np.array_equal(m, want_m) and np.array_equal(s, want_s), rank


def _gpu_worker(rank, world, port, images, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "arm-neon-opencv_amd"))
    import torch.distributed as dist
    from vacv_amd import ops
    from vacv_amd.dist import allreduce_sums, shard_range, stats_from_moments
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")  # both ranks on the one card of the box
    b, e = shard_range(len(images), rank, world)
    shard = torch.from_numpy(np.stack(images[b:e])).to(dev)
    # vacv_channel_sums of this rank's shard on the GPU, all-reduced
    local = ops.channel_sums(shard, per_image=False)[0].cpu()
    h, w = images[0].shape[:2]
    total, count = allreduce_sums(local, float((e - b) * h * w))
    mean, std = stats_from_moments(total, count)
    # the single-process answer: the whole batch on this rank's GPU
    full = ops.channel_sums(torch.from_numpy(np.stack(images)).to(dev), per_image=False)[0].cpu()
    fm, fs = stats_from_moments(full, float(len(images) * h * w))
    out_q.put((rank, mean.numpy(), std.numpy(), count, bool(torch.equal(total, full)),
               bool(torch.equal(mean, fm) and torch.equal(std, fs))))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_global_stats_two_ranks_on_gpu():
    """The exchange step on real kernels: two ranks (gloo, both on cuda:0)
    each reduce their shard with vacv_channel_sums on the GPU and all-reduce
    the fp64 sums; the result equals the whole batch's sums on one rank
    (exact: integer-valued fp64) and the oracle's exact mean / stddev."""
    from oracle import Oracle, synthetic_image
    images = [synthetic_image(700 + k, 90, 160, 3) for k in range(7)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, images, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    O = Oracle()
    want_m, want_s = O.mean_stddev_exact(np.concatenate([im.reshape(-1, 3) for im in images])[None])
    for rank, m, s, count, same_sums, same_stats in res:
        assert count == 7 * 90 * 160
        assert same_sums and same_stats, rank
        assert np.array_equal(m, want_m) and np.array_equal(s, want_s), rank
