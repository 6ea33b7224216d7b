"""CPU, world_size 2 over gloo: the flat-buffer gradient bucketer (the RCCL path's logic) produces
exactly the rank-averaged gradients DDP would, with several buckets and readiness driven by
autograd post-accumulate hooks; rank-0 parameter broadcast matches DDP's constructor."""

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.GELU(), torch.nn.Linear(64, 64), torch.nn.GELU(),
                               torch.nn.Linear(64, 4))


def _grads(model, x):
    model.zero_grad()
    model(x).pow(2).sum().backward()
    return torch.cat([p.grad.flatten() for p in model.parameters()])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__

    __graft_entry__.load_package()
    from spine_vision_amd.training.comm import GradBucketer, broadcast_parameters
    from spine_vision_amd.training.flat import FlatArena

    model = _model(seed=100 + rank)  # different init per rank -> broadcast must fix it
    arena = FlatArena(model, "cpu", with_shadow=False)
    broadcast_parameters(arena, model)
    ref0 = _model(seed=100)
    ok_bcast = all(torch.equal(a, b) for a, b in zip(model.parameters(), ref0.parameters()))
    buck = GradBucketer(arena, bucket_mb=4096 * 4 / 1024 / 1024)  # ~4K floats per bucket -> several buckets
    buck.attach(model)
    xs = [torch.randn(8, 16, generator=torch.Generator().manual_seed(7 + r)) for r in range(world)]
    arena.zero_grad()
    model(xs[rank]).pow(2).sum().backward()
    buck.finish()
    got = torch.cat([p.grad.flatten() for p in model.parameters()])
    expect = sum(_grads(_model(seed=100), x) for x in xs) / world
    q.put((rank, ok_bcast, len(buck.buckets), float((got - expect).abs().max())))
    dist.destroy_process_group()


def test_bucketed_allreduce_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_bcast, nb, err in res:
        assert ok_bcast
        assert nb >= 2
        assert err < 1e-5, (rank, err)


def _bn_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__

    __graft_entry__.load_package()
    from spine_vision_amd.training.comm import BufferSync

    torch.manual_seed(rank)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.ReLU(),
                                torch.nn.Conv2d(8, 8, 1), torch.nn.BatchNorm2d(8))
    model.train()
    sync = BufferSync(model)
    ok = True
    for step in range(3):
        sync.sync()  # DDP broadcast_buffers: rank 0's running stats before every forward
        got = torch.cat([model[1].running_mean, model[1].running_var, model[4].running_mean, model[4].running_var])
        all_ = [torch.empty_like(got) for _ in range(world)]
        dist.all_gather(all_, got)
        ok &= all(torch.equal(all_[0], a) for a in all_)
        # each rank sees different data -> running stats diverge until the next sync
        model(torch.randn(4, 3, 8, 8, generator=torch.Generator().manual_seed(10 * step + rank)))
    ok &= model[1].running_mean.data_ptr() == sync.flat.data_ptr()  # still bound to the flat buffer
    q.put((rank, ok, int(model[1].num_batches_tracked)))
    dist.destroy_process_group()


def test_bn_buffer_broadcast_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bn_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, nbt in res:
        assert ok, rank
        assert nbt == 3


def _split_report_worker(rank, world, port, q):
    """Readiness reported the way ConvNeXt reports it: one bucket's parameters in two separate mark_ready calls
    (block weights from the side stream, then the downsample from the main stream), the last report closing the
    bucket exactly on its lowest parameter (the 'downsample').  On CPU there are no streams; this pins the bookkeeping
    (pending counts per report, a bucket launched once, when its last parameter reports) that the GPU test
    test_ddp_gpu.py::test_two_rank_bucket_ending_on_downsample_waits_for_every_stream runs with real streams."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__

    __graft_entry__.load_package()
    from spine_vision_amd.training.comm import GradBucketer
    from spine_vision_amd.training.flat import FlatArena, _align

    model = _model(seed=100)
    ps = list(model.parameters())  # [l0.w, l0.b, l1.w, l1.b, l2.w, l2.b]; "downsample" = l1.w
    bucket_mb = sum(_align(p.numel()) for p in ps[2:]) * 4 / 2**20
    arena = FlatArena(model, "cpu", with_shadow=False)
    buck = GradBucketer(arena, bucket_mb=bucket_mb)
    first = buck.buckets[0]
    ends_on_ds = arena.params[first[2][-1]] is ps[2]
    x = torch.randn(8, 16, generator=torch.Generator().manual_seed(7 + rank))
    arena.zero_grad()
    model(x).pow(2).sum().backward()
    buck.mark_ready([ps[5], ps[4], ps[3]])  # the "side stream" block report
    launched_early = buck.launched[0]
    buck.mark_ready([ps[2]])  # the "main stream" downsample report closes the bucket
    launched_on_last = buck.launched[0]
    buck.mark_ready([ps[3], ps[2]])  # repeated reports are ignored
    buck.finish()
    got = torch.cat([p.grad.flatten() for p in model.parameters()])
    xs = [torch.randn(8, 16, generator=torch.Generator().manual_seed(7 + r)) for r in range(world)]
    expect = sum(_grads(_model(seed=100), xx) for xx in xs) / world
    q.put((rank, ends_on_ds, launched_early, launched_on_last, float((got - expect).abs().max())))
    dist.destroy_process_group()


def test_bucket_closed_by_a_split_report_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_split_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ends_on_ds, early, on_last, err in res:
        assert ends_on_ds and not early and on_last, (rank, ends_on_ds, early, on_last)
        assert err < 1e-5, (rank, err)
