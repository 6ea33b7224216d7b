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
