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


def _rccl_worker(port, images, out_q):
    """One rank over the "nccl" backend (RCCL on ROCm), in a fresh process:
    the cfg5 exchange exactly as bench.py's cubic_stats step runs it --
    vacv_channel_sums of the shard on the device, all_reduce(SUM) of the fp64
    device tensor over RCCL, vacv_stats_from_sums -- with no host round trip."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "arm-neon-opencv_amd"))
    try:
        import torch.distributed as dist
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from vacv_amd import ops
        backend = dist.get_backend()
        batch = torch.from_numpy(np.stack(images)).to(dev)
        local = ops.channel_sums(batch, per_image=False)  # (1, c, 2) fp64 on the device
        sums = local.clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        h, w = images[0].shape[:2]
        mean, std = ops.stats_from_sums(sums, float(len(images) * h * w))
        torch.cuda.synchronize()
        out_q.put((backend, str(sums.device), bool(torch.equal(sums, local)), sums.cpu().numpy(),
                   mean.cpu().numpy(), std.cpu().numpy()))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the parent on q.get
        out_q.put(("error", repr(e)))
        raise


@pytest.mark.gpu
def test_global_stats_rccl_one_rank():
    """The design's only collective (cfg5's global mean/stddev)
    on RCCL itself: init_process_group("nccl") in a freshly spawned process,
    all_reduce of vacv_channel_sums' fp64 device output, vacv_stats_from_sums.
    At world size 1 the all-reduce must return the local sums unchanged, and
    the statistics must equal the oracle's exact mean / stddev bit for bit."""
    from oracle import Oracle, synthetic_image
    images = [synthetic_image(710 + k, 96, 160, 3) for k in range(5)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), images, q))
    p.start()
    res = q.get(timeout=180)
    p.join(timeout=60)
    assert res[0] != "error", res
    assert p.exitcode == 0
    backend, device, unchanged, sums, mean, std = res
    assert backend == "nccl" and device == "cuda:0"
    assert unchanged, "all_reduce at world size 1 changed the sums"
    O = Oracle()
    flat = np.concatenate([im.reshape(-1, 3) for im in images])
    assert np.array_equal(sums.reshape(-1), O.channel_sums(flat[None])), "sums exact"
    want_m, want_s = O.mean_stddev_exact(flat[None])
    assert np.array_equal(mean[0], want_m) and np.array_equal(std[0], want_s)


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


def _bench_rank_worker(rank, world, port, batch, out_q):
    """One rank of bench.py's cfg5 step on cuda:0 (gloo): make_workload's
    main + extra exactly as bench.py runs them at world > 1 -- the fused
    device sums of this rank's shard, the all-reduce, vacv_stats_from_sums."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (repo, os.path.join(repo, "arm-neon-opencv_amd")):
        sys.path.insert(0, p)
    try:
        import torch.distributed as dist
        import bench
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda:0")  # both ranks on the one card of the box
        torch.cuda.set_device(dev)
        from vacv_amd import ops
        wl = bench.make_workload("cubic_stats", batch, dev, rank, world, ops)
        for _ in range(2):  # a repeated step gives the same answer
            wl["main"]()
            wl["extra"]()
        torch.cuda.synchronize(dev)
        st = wl["stats"]
        out_q.put((rank, st["sums"].cpu().numpy(), st["mean"].cpu().numpy(), st["std"].cpu().numpy()))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the parent on q.get
        out_q.put(("error", repr(e)))
        raise


@pytest.mark.gpu
def test_bench_cubic_stats_two_ranks(hip_device):
    """bench.py --workload cubic_stats at world size 2, on real kernels: two
    spawned gloo ranks on cuda:0 run make_workload's main + extra as the bench
    does (fused cubic sums per rank, all-reduce of the device sums, stats).
    Both ranks agree bit for bit, and their global mean / stddev equal one
    process running the whole batch (vacv_resize_mean_stddev) within SURVEY
    8(c)'s |d mean| <= 1e-3, |d std| / std <= 1e-4."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from vacv_amd import INTER_CUBIC, ops
    batch = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_rank_worker, args=(r, 2, port, batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "error" for r in res), res
    assert all(p.exitcode == 0 for p in procs)
    res.sort(key=lambda r: r[0])
    (_, s0, m0, d0), (_, s1, m1, d1) = res
    assert np.array_equal(s0, s1) and np.array_equal(m0, m1) and np.array_equal(d0, d1), "ranks disagree"
    # the whole batch in one process: both ranks' inputs, regenerated the way
    # make_workload draws them (seed 1234 + rank on this device)
    dev = hip_device
    whole = torch.cat([bench.make_workload("cubic_stats", batch, dev, r, 2, ops)["inputs"] for r in range(2)])
    _, sums, mean, std = ops.resize_mean_stddev(whole, 224, 224, INTER_CUBIC, per_image=False)
    torch.cuda.synchronize(dev)
    sums, mean, std = sums.cpu().numpy(), mean.cpu().numpy(), std.cpu().numpy()
    assert np.abs(s0 - sums).max() / np.abs(sums).max() <= 1e-12
    assert np.abs(m0 - mean).max() <= 1e-3
    assert (np.abs(d0 - std) / std).max() <= 1e-4
    del whole
    torch.cuda.empty_cache()
