"""CPU, world_size 2 over gloo: the trainer's multi-process host logic.

* validation with a val set that is NOT a multiple of batch x world: every rank yields the same
  number of full batches (accelerate's even_batches padding), the per-batch all-gather of
  ``LocalizationTrainer._validate_epoch`` completes and both ranks compute the same metrics over
  world x batches x batch_size gathered rows (the reference's ``accelerator.gather`` keeps the
  padded duplicates: trainers/localization.py:240-242);
* the cosine T_max counts the unsharded loader (reference base.py:243-266: the scheduler is built
  before ``accelerator.prepare``), so at world 2 it equals the single-process value.
"""

import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import __graft_entry__

    __graft_entry__.load_package()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from test_trainer_cpu import CpuLocTrainer, TinyLoc, _cfg

    from spine_vision_amd.training.datasets import SyntheticLocalizationDataset

    torch.manual_seed(0)
    cfg = _cfg(tmp, num_epochs=3, batch_size=4)
    tr = CpuLocTrainer(cfg, model=TinyLoc(), train_dataset=SyntheticLocalizationDataset(37, (32, 32), seed=1),
                       val_dataset=SyntheticLocalizationDataset(10, (32, 32), seed=2))
    n_val_batches = len(tr.val_loader)
    rows = []
    orig = tr._gather

    def counting_gather(t):
        out = orig(t)
        rows.append(out.shape[0])
        return out

    tr._gather = counting_gather
    val_loss, metrics = tr._validate_epoch()
    q.put((rank, tr.world, tr.scheduler.T_max, n_val_batches, sum(rows) // 3, {k: float(v) for k, v in metrics.items()}))
    dist.destroy_process_group()


def test_validation_and_scheduler_gloo_world2(tmp_path):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path / f"r{r}"), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # 10 val samples, bs 4, world 2: unsharded batches [4,4,2] -> 2 full batches per rank (padded)
    for rank, w, tmax, nvb, nrows, metrics in res:
        assert w == 2
        assert tmax == (37 // 4) * 3  # unsharded: 9 batches x 3 epochs
        assert nvb == 2
        assert nrows == world * nvb * 4
    assert res[0][5] == res[1][5]  # identical gathered metrics on both ranks
