"""Trainer host -- drop-in for spine_vision/training/trainers/base.py (TrainingConfig 41-162,
TrainingResult 165-175, BaseTrainer 194-805).

Same configuration fields/defaults, same epoch loop, history, validation, LR scheduling, checkpoint
dict and files, early stopping and hooks.  What changes is the step: instead of accelerate
(DDP + GradScaler + foreach AdamW) the default optimizer is the flat-buffer ``FlatAdamW`` and the
step is ``StepEngine``-style: one gradient memset, HIP backbone fwd/bwd, RCCL bucket all-reduce
overlapped with the backward on a side stream, device-side clip coefficient, fused AdamW.  The
per-step ``loss.item()`` host sync of the reference (base.py:599) is deferred to logging points.

Reference quirks kept on purpose: cosine T_max counted in steps but stepped once per
epoch, ``num_processes`` times per call (accelerate's AcceleratedScheduler); ``history`` replaced by
the best checkpoint's at the end of ``train()``; seed set after model construction.
Multi-process: one process per GPU (``torchrun`` / ``accelerate launch`` env vars), "nccl" (RCCL)
on GPU, "gloo" on CPU; batches sharded like accelerate's BatchSamplerShard (rank r takes every
world-th batch of one shared sampler stream).
"""

from __future__ import annotations

import logging
import os
import random
import uuid
from dataclasses import dataclass, field
from datetime import datetime
from pathlib import Path
from typing import Any, Literal

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
from pydantic import BaseModel, ConfigDict, model_validator
from torch.utils.data import DataLoader, Dataset, Sampler

from .. import optim as flat_optim
from ..comm import BufferSync, GradBucketer, broadcast_parameters
from ..engine import InflightLimiter
from ..flat import FlatArena

logger = logging.getLogger("spine_vision_amd")


class BaseConfig(BaseModel):
    """spine_vision/core/config.py:8-15."""

    verbose: bool = False
    enable_file_log: bool = False
    log_path: Path = Path.cwd() / "logs"
    model_config = ConfigDict(arbitrary_types_allowed=True)


def generate_run_id() -> str:
    return f"{datetime.now().strftime('%Y%m%d_%H%M%S')}_{uuid.uuid4().hex[:6]}"


class TrainingConfig(BaseConfig):
    run_id: str = ""
    task: str = "training"
    data_path: Path = Path("data/processed/localization")
    output_path: Path | None = None
    checkpoint_path: Path | None = None
    batch_size: int = 32
    num_epochs: int = 15
    learning_rate: float = 1e-4
    weight_decay: float = 1e-5
    grad_clip: float | None = 1.0
    scheduler_type: Literal["cosine", "step", "plateau", "none"] = "cosine"
    scheduler_patience: int = 10
    scheduler_step_size: int = 30
    scheduler_gamma: float = 0.1
    warmup_epochs: int = 5
    early_stopping: bool = True
    patience: int = 20
    min_delta: float = 1e-4
    val_split: float = 0.2
    val_frequency: int = 1
    device: str = "cuda:0"
    num_workers: int = 4
    pin_memory: bool = True
    mixed_precision: bool = True
    log_frequency: int = 10
    save_frequency: int = 10
    use_trackio: bool = False
    use_space: bool = True
    trackio_project: str = "spine-vision"
    trackio_run_name: str | None = None
    seed: int = 42
    # MI355X build additions
    precision: Literal["bf16", "fp32"] = "bf16"
    """Backbone compute precision: bf16 MFMA (throughput; the reference's fp16 autocast analogue) or
    exact f32 MFMA (parity with the reference CPU path).  ``mixed_precision=False`` forces fp32."""
    bucket_mb: float = 64.0
    """Gradient all-reduce bucket size (MB) for multi-GPU runs."""
    device_transform: bool = False
    """Input pipeline (row f1): datasets yield decoded uint8 images and the reference transform tail
    (ToTensor -> Normalize) runs on the GPU.  Localization: uint8 grayscale [H,W], RGB-replicated and
    normalised inside the ConvNeXt stem's patch gather (bf16) or by ``sv_normalize_u8_gray`` (fp32) --
    12x fewer host->device bytes.  Classification: the uint8 [H,W,3] crop of construct_3channel
    ([T2,T1,T2] or one plane replicated), normalised inside the ResNet stem's NHWC conversion
    (``sv_image_u8_hwc_to_nhwc``) -- 4x fewer bytes.  No per-sample float work in the workers."""

    model_config = {"arbitrary_types_allowed": True}

    @model_validator(mode="after")
    def setup_paths(self) -> "TrainingConfig":
        if not self.run_id:
            object.__setattr__(self, "run_id", generate_run_id())
        if self.output_path is None:
            object.__setattr__(self, "output_path", Path("weights") / self.task / self.run_id)
        if self.use_trackio and self.trackio_run_name is None:
            object.__setattr__(self, "trackio_run_name", self.run_id)
        return self

    @property
    def effective_precision(self) -> str:
        return self.precision if self.mixed_precision else "fp32"

    @property
    def logs_path(self) -> Path:
        return self.output_path / "logs"

    @property
    def config_path(self) -> Path:
        return self.output_path / "config.yaml"

    def save_config(self) -> None:
        import yaml

        self.output_path.mkdir(parents=True, exist_ok=True)
        d = {k: (str(v) if isinstance(v, Path) else v) for k, v in self.model_dump().items()}
        with open(self.config_path, "w") as f:
            yaml.dump(d, f, default_flow_style=False, sort_keys=False)


@dataclass
class TrainingResult:
    best_epoch: int
    best_metric: float
    final_train_loss: float
    final_val_loss: float
    history: dict[str, list[float]] = field(default_factory=dict)
    checkpoint_path: Path | None = None
    metadata: dict[str, Any] = field(default_factory=dict)


@dataclass
class EpochResult:
    epoch: int
    train_loss: float
    val_loss: float | None = None
    metrics: dict[str, float] = field(default_factory=dict)
    lr: float = 0.0


class ShardedBatchSampler(Sampler):
    """accelerate's BatchSamplerShard (split_batches=False, even_batches=True -- the default that
    ``accelerator.prepare`` builds for the reference's train and val loaders, base.py:253-263):
    batches of the underlying sampler are dealt round-robin to the ranks.  With ``drop_last`` an
    incomplete final group is cut; without it (validation) the last group is completed by cycling
    indices from the start of the epoch, so every rank yields the same number of FULL batches and the
    per-batch all-gather of ``_validate_epoch`` always sees equal shapes (the duplicated samples are
    then part of the gathered metrics, exactly as with the reference's ``accelerator.gather``)."""

    def __init__(self, sampler, batch_size: int, drop_last: bool, rank: int, world: int) -> None:
        self.sampler, self.batch_size, self.drop_last = sampler, batch_size, drop_last
        self.rank, self.world = rank, world

    def _batches(self):
        b = []
        for i in self.sampler:
            b.append(i)
            if len(b) == self.batch_size:
                yield b
                b = []
        if b and not self.drop_last:
            yield b

    def __iter__(self):
        if self.world == 1:  # accelerate does not shard (or pad) a single-process loader
            yield from self._batches()
            return
        bs, world, rank = self.batch_size, self.world, self.rank
        head: list = []  # indices of the first `world` batches: the padding source
        pending = None
        idx, last = -1, []
        for idx, b in enumerate(self._batches()):
            if not self.drop_last and idx < world:
                head += b
            if idx % world == rank:
                pending = b
            if idx % world == world - 1 and len(b) == bs:
                yield pending
                pending = None
            last = b
        if self.drop_last or not head:
            return
        if pending is not None and len(pending) == bs:
            yield pending
        while len(head) < world * bs:  # fewer samples than one full group
            head = head + head
        batch = list(last)
        if len(batch) == bs:  # the last batch was full and went out with its group
            batch, idx = [], idx + 1
        pos = 0
        while idx % world != 0 or batch:
            take = bs - len(batch)
            batch = batch + head[pos : pos + take]
            if idx % world == rank:
                yield batch
            pos += take
            batch, idx = [], idx + 1

    def num_batches(self) -> int:
        """Batches per epoch of the UNSHARDED loader (what the reference's scheduler counts)."""
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __len__(self) -> int:
        nb = self.num_batches()
        if self.world == 1 or nb % self.world == 0 or self.drop_last:
            return nb // self.world
        return nb // self.world + 1


class BaseTrainer:
    def __init__(self, config: TrainingConfig, model: nn.Module, train_dataset: Dataset,
                 val_dataset: Dataset | None = None) -> None:
        self.config = config
        self.train_dataset, self.val_dataset = train_dataset, val_dataset
        self._setup_distributed()
        self.model = model.to(self.device)
        self.train_loader = self._create_dataloader(train_dataset, shuffle=True)
        self.val_loader = self._create_dataloader(val_dataset, shuffle=False) if val_dataset else None
        self.optimizer = self._create_optimizer()
        self.scheduler = self._create_scheduler()
        self.bucketer = None
        self.buffer_sync = None
        # bounded host lookahead (engine.InflightLimiter): side-stream tensors of queued steps stay pinned
        self._limiter = InflightLimiter() if self.device.type == "cuda" else None
        if self.world > 1:
            self.buffer_sync = BufferSync(self.model)
            if isinstance(self.optimizer, flat_optim.FlatAdamW):
                broadcast_parameters(self.optimizer.arena, self.model)
                self.bucketer = GradBucketer(self.optimizer.arena, bucket_mb=config.bucket_mb)
                self.bucketer.attach(self.model)
            else:  # generic optimizer: DDP semantics by flat all-reduce after backward
                for p in self.model.parameters():
                    dist.broadcast(p.data, 0)
        self.current_epoch = 0
        self.best_metric = float("inf")
        self.best_epoch = 0
        self.patience_counter = 0
        self.history: dict[str, list[float]] = {"train_loss": [], "val_loss": [], "lr": []}
        self.config.output_path.mkdir(parents=True, exist_ok=True)
        self.config.logs_path.mkdir(parents=True, exist_ok=True)
        if self.is_main_process:
            self.config.save_config()
        self._set_seed(config.seed)

    # -- process / device ---------------------------------------------------------------------
    def _setup_distributed(self) -> None:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world > 1 and not (dist.is_available() and dist.is_initialized()):
            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
            dist.init_process_group(backend)
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        if torch.cuda.is_available():
            self.device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        else:
            self.device = torch.device("cpu")

    @property
    def is_main_process(self) -> bool:
        return self.rank == 0

    def _set_seed(self, seed: int) -> None:
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)

    # -- factories (override points, as in the reference) ----------------------------------------
    def _collate_fn(self):
        return None

    def _sampler(self, dataset: Dataset, shuffle: bool):
        if shuffle:
            g = torch.Generator()
            g.manual_seed(self.config.seed)
            return torch.utils.data.RandomSampler(dataset, generator=g)
        return torch.utils.data.SequentialSampler(dataset)

    def _create_dataloader(self, dataset: Dataset, shuffle: bool = True) -> DataLoader:
        sampler = self._sampler(dataset, shuffle)
        bs = ShardedBatchSampler(sampler, self.config.batch_size, drop_last=shuffle, rank=self.rank, world=self.world)
        return DataLoader(dataset, batch_sampler=bs, num_workers=self.config.num_workers,
                          pin_memory=self.config.pin_memory and self.device.type == "cuda",
                          collate_fn=self._collate_fn())

    def _create_optimizer(self) -> torch.optim.Optimizer:
        """Flat-buffer fused AdamW on the MI355X (torch AdamW semantics: lr, betas (0.9,0.999),
        eps 1e-8, weight_decay on every parameter).  Override for custom optimizers."""
        arena = FlatArena(self.model, self.device, with_shadow=True)
        return flat_optim.FlatAdamW(arena, lr=self.config.learning_rate, weight_decay=self.config.weight_decay)

    def _create_scheduler(self):
        c = self.config
        if c.scheduler_type == "none":
            return None
        # the reference builds the scheduler BEFORE accelerator.prepare shards the loader (base.py:243-266),
        # so T_max counts the unsharded batches; _scheduler_step then steps it world times per epoch
        bsamp = getattr(self.train_loader, "batch_sampler", None)
        per_epoch = bsamp.num_batches() if isinstance(bsamp, ShardedBatchSampler) else len(self.train_loader)
        total = per_epoch * c.num_epochs
        if c.scheduler_type == "cosine":
            return torch.optim.lr_scheduler.CosineAnnealingLR(self.optimizer, T_max=total, eta_min=c.learning_rate * 0.01)
        if c.scheduler_type == "step":
            return torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=c.scheduler_step_size, gamma=c.scheduler_gamma)
        return torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer, mode="min", factor=c.scheduler_gamma,
                                                          patience=c.scheduler_patience)

    def _scheduler_step(self, val_loss: float | None) -> None:
        if self.scheduler is None:
            return
        if isinstance(self.scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
            if val_loss is not None:
                self.scheduler.step(val_loss)
            return
        for _ in range(self.world):  # accelerate's AcceleratedScheduler steps num_processes times
            self.scheduler.step()

    # -- the step ------------------------------------------------------------------------------
    def _optimize(self, loss_fn) -> torch.Tensor:
        """zero_grad -> forward/loss -> backward (+bucketed all-reduce) -> clip -> optimizer step."""
        opt = self.optimizer
        opt.zero_grad()
        if self.buffer_sync is not None:
            self.buffer_sync.sync()
        loss = loss_fn()
        loss.backward()
        if isinstance(opt, flat_optim.FlatAdamW):
            if self.bucketer is not None:
                self.bucketer.finish()
            scale = None
            if self.config.grad_clip:
                from ... import kernels as K

                scale = K.grad_clip_coef(opt.arena.grad_flat, self.config.grad_clip)[1:2]
            opt.step(grad_scale=scale)
            if self._limiter is not None:
                self._limiter.step_done()
        else:
            params = [p for p in self.model.parameters() if p.grad is not None]
            if self.world > 1:
                for p in params:
                    dist.all_reduce(p.grad)
                    p.grad.div_(self.world)
            if self.config.grad_clip:
                torch.nn.utils.clip_grad_norm_(params, self.config.grad_clip)
            opt.step()
        return loss.detach()

    def _train_step(self, batch: Any) -> torch.Tensor:
        inputs, targets = self._unpack_batch(batch)
        inputs = inputs.to(self.device, non_blocking=True)
        return self._optimize(lambda: self.model.get_loss(self.model(inputs), targets.to(self.device)))

    def _unpack_batch(self, batch: Any):
        raise NotImplementedError

    def _compute_metrics(self, predictions, targets) -> dict[str, float]:
        return {}

    # -- loop ----------------------------------------------------------------------------------
    def train(self) -> TrainingResult:
        logger.info("Starting training for %d epochs (%s, %d process(es), precision %s)", self.config.num_epochs,
                    getattr(self.model, "name", "Model"), self.world, self.config.effective_precision)
        if self.config.checkpoint_path:
            self._load_checkpoint(self.config.checkpoint_path)
        self.on_train_begin()
        for epoch in range(self.current_epoch, self.config.num_epochs):
            self.current_epoch = epoch
            self.on_epoch_begin(epoch)
            train_loss = self._train_epoch()
            self.history["train_loss"].append(train_loss)
            self.history["lr"].append(self.optimizer.param_groups[0]["lr"])
            val_loss, metrics = None, {}
            if self.val_loader is not None and (epoch + 1) % self.config.val_frequency == 0:
                val_loss, metrics = self._validate_epoch()
                self.history["val_loss"].append(val_loss)
                for k, v in metrics.items():
                    self.history.setdefault(k, []).append(v)
            self._scheduler_step(val_loss)
            self._log_epoch(epoch, train_loss, val_loss, metrics)
            self.on_epoch_end(epoch, {"train_loss": train_loss, "val_loss": val_loss, **metrics})
            m = self.get_metric_for_checkpoint(val_loss, metrics)
            if m < self.best_metric - self.config.min_delta:
                self.best_metric, self.best_epoch, self.patience_counter = m, epoch, 0
                self._save_checkpoint(is_best=True)
            else:
                self.patience_counter += 1
            if (epoch + 1) % self.config.save_frequency == 0:
                self._save_checkpoint(is_best=False)
            if self.config.early_stopping and self.patience_counter >= self.config.patience:
                logger.info("Early stopping at epoch %d", epoch + 1)
                break
        best = self.config.output_path / "best_model.pt"
        if self.world > 1:
            dist.barrier()
        if best.exists():
            self._load_checkpoint(best)
        result = TrainingResult(best_epoch=self.best_epoch, best_metric=self.best_metric,
                                final_train_loss=self.history["train_loss"][-1],
                                final_val_loss=self.history["val_loss"][-1] if self.history["val_loss"] else 0.0,
                                history=self.history, checkpoint_path=best)
        self.on_train_end(result)
        return result

    def _train_epoch(self) -> float:
        self.model.train()
        total = torch.zeros((), device=self.device, dtype=torch.float64)
        n = 0
        for i, batch in enumerate(self.train_loader):
            total += self._train_step(batch).double()
            n += 1
            if (i + 1) % self.config.log_frequency == 0:
                logger.debug("Epoch %d [%d/%d] Loss: %.6f", self.current_epoch, i + 1, len(self.train_loader),
                             float(total) / n)
        return float(total) / max(n, 1)

    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t.contiguous())
        return torch.cat(out, 0)

    def _validate_epoch(self) -> tuple[float, dict[str, float]]:
        self.model.eval()
        total, n = 0.0, 0
        preds, tgts = [], []
        with torch.no_grad():
            for batch in self.val_loader:
                inputs, targets = self._unpack_batch(batch)
                p = self.model(inputs.to(self.device))
                total += float(self.model.get_loss(p, targets.to(self.device)))
                n += 1
                preds.append(self._gather(p).cpu())
                tgts.append(self._gather(targets.to(self.device)).cpu())
        metrics = self._compute_metrics(torch.cat(preds), torch.cat(tgts)) if preds else {}
        return total / max(n, 1), metrics

    def _log_epoch(self, epoch, train_loss, val_loss, metrics) -> None:
        msg = f"Epoch {epoch + 1}/{self.config.num_epochs} - Train Loss: {train_loss:.6f}"
        if val_loss is not None:
            msg += f" - Val Loss: {val_loss:.6f}"
        for k, v in metrics.items():
            msg += f" - {k}: {v:.4f}"
        msg += f" - LR: {self.optimizer.param_groups[0]['lr']:.2e}"
        logger.info(msg)

    # -- checkpoints (dict keys as base.py:695-706; timm/state_dict key names) -----------------------
    def _save_checkpoint(self, is_best: bool = False) -> None:
        if not self.is_main_process:
            return
        ck = {
            "epoch": self.current_epoch,
            "model_state_dict": self.model.state_dict(),
            "optimizer_state_dict": self.optimizer.state_dict(),
            "scheduler_state_dict": self.scheduler.state_dict() if self.scheduler else None,
            "best_metric": self.best_metric,
            "best_epoch": self.best_epoch,
            "history": self.history,
            "config": self.config.model_dump(),
        }
        path = self.config.output_path / ("best_model.pt" if is_best else f"checkpoint_epoch_{self.current_epoch + 1}.pt")
        torch.save(ck, path)

    def _load_checkpoint(self, path: Path) -> None:
        # our own checkpoints contain only tensors, numbers, strings and Paths
        import pathlib

        with torch.serialization.safe_globals([pathlib.PosixPath, pathlib.Path]):
            ck = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ck["model_state_dict"])
        self.optimizer.load_state_dict(ck["optimizer_state_dict"])
        if isinstance(self.optimizer, flat_optim.FlatAdamW):
            self.optimizer.arena.refresh_shadow()
        if self.scheduler and ck["scheduler_state_dict"]:
            self.scheduler.load_state_dict(ck["scheduler_state_dict"])
        self.current_epoch = ck["epoch"] + 1
        self.best_metric = ck["best_metric"]
        self.best_epoch = ck["best_epoch"]
        self.history = ck["history"]

    # -- hooks ---------------------------------------------------------------------------------
    def on_train_begin(self) -> None:
        pass

    def on_epoch_begin(self, epoch: int) -> None:
        pass

    def on_epoch_end(self, epoch: int, metrics: dict[str, float]) -> None:
        pass

    def on_train_end(self, result: TrainingResult) -> None:
        pass

    def get_metric_for_checkpoint(self, val_loss: float | None, metrics: dict[str, float]) -> float:
        if val_loss is not None:
            return val_loss
        return self.history["train_loss"][-1] if self.history["train_loss"] else float("inf")
