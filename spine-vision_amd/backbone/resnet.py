"""ResNet-18 / ResNet-50 backbone on the gfx950 kernel library -- drop-in for
``timm.create_model("resnet18.a1_in1k" | "resnet50.a1_in1k", num_classes=0)`` as called at
spine_vision/training/models/backbone.py:166-170 (names at backbone.py:27,29; timm 1.0.22
``timm/models/resnet.py``: BasicBlock [2,2,2,2] / Bottleneck [3,4,6,3], stride on the 3x3 conv,
1x1 conv + BN downsample, conv7x7/s2 stem + BN + ReLU + MaxPool(3,2,1), global average pool).

* Same module tree / ``state_dict`` keys as timm (``conv1``, ``bn1``, ``layerN.i.{conv1,bn1,conv2,bn2,
  conv3,bn3,downsample.{0,1}}``), ``num_features``, ``forward([B,3,H,W] f32) -> [B,F]``.  Sub-modules
  are parameter/buffer containers; their own ``forward`` is never called.
* Every convolution is an implicit GEMM on MFMA over NHWC activations (``sv_conv_*``; no im2col
  buffers); BatchNorm uses train-mode batch statistics (and updates running_mean / running_var /
  num_batches_tracked exactly like torch) or the running statistics in eval mode; BN + ReLU (+ the
  residual add, including the BN of the downsample shortcut) is one fused pass.
* Backward is an explicit kernel sequence writing the parameter gradients into ``p.grad`` (views of
  the trainer's flat gradient buffer) and calling ``grad_ready_hook`` after each block so the DDP
  bucketer can start all-reducing while earlier blocks are still being differentiated.
* ``precision="bf16"``: bf16 MFMA, bf16 activations and a bf16 gradient stream (the block output / input
  gradients, as under the reference's fp16 autocast: ``batch_norm`` is not on autocast's fp32 list, so its
  inputs, outputs and gradients are 16-bit there -- VERDICT r4, weak 8); f32 statistics, accumulation and master
  weights.  ``precision="fp32"``: f32 everywhere with exact f32 MFMA (parity mode).
"""

from __future__ import annotations

import os
import weakref
from dataclasses import dataclass, field
from typing import Callable

import torch
import torch.nn as nn

from .. import kernels as K
from .. import native as nv

# SV_MULTI_PACK=0: one weight-pack launch per conv in the forward (A/B runs)
_MULTI_PACK = os.environ.get("SV_MULTI_PACK", "1") != "0"
# SV_POOLED_STEM_BWD=0: the max-pool backward as its own pass before the stem BatchNorm's (A/B runs)
_POOLED_STEM_BWD = os.environ.get("SV_POOLED_STEM_BWD", "1") != "0"
# SV_FIRST_BLOCK_SIDE=0: the first block's weight gradients on the main stream (A/B runs)
_FIRST_BLOCK_SIDE = os.environ.get("SV_FIRST_BLOCK_SIDE", "1") != "0"
# SV_DEFER_WGRAD_FLUSH=1: a block's side-stream weight gradients are enqueued after the NEXT block's first BatchNorm
# backward pass, so the main queue has work while the host enqueues them (the traced step's largest main-queue idle
# sits before each block's first BatchNorm pass, r16b); same kernels and operands, so the same bits
_DEFER_FLUSH = os.environ.get("SV_DEFER_WGRAD_FLUSH", "0") == "1"
# SV_BN_BWD_EPI: the inner BatchNorms' backward statistics from the split-K finish of their data gradient
# (split, default: +2.2 %), also from the unsplit GEMMs' epilogue (1: no faster than a separate pass, the
# layer1/2 epilogues absorb what the pass saved), or from their own pass everywhere (0) -- r6e A/B
_BN_BWD_EPI = os.environ.get("SV_BN_BWD_EPI", "split")
# SV_S2_BN=1: the strided 3x3s' inner BatchNorm statistics from the one-launch parity-class dgrad's
# epilogue (SV_EPI_STORE_BN_BWD) instead of their own pass: -0.9 % (r9i, as for stride 1)
_S2_BN = os.environ.get("SV_S2_BN", "0") == "1"
# SV_BN_DUAL=0: a projection-shortcut block's two output BatchNorm backwards as separate passes (A/B runs)
_BN_DUAL = os.environ.get("SV_BN_DUAL", "1") != "0"
# SV_RESNET_GRAD_BF16=0: the bf16 model's gradient stream (block output / input gradients) in f32 (A/B runs; the
# round-4 layout)
_GRAD_BF16 = os.environ.get("SV_RESNET_GRAD_BF16", "1") != "0"

RESNET_CFGS = {"resnet18": ("basic", (2, 2, 2, 2)), "resnet50": ("bottleneck", (3, 4, 6, 3))}
_MAX_FORWARD_GRAPHS = 8  # captured forward graphs per model (input signatures beyond that run eagerly)
BN_EPS = 1e-5


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def convs(self):
        """(conv, bn, kernel, stride, pad, relu) of the main path, in forward order."""
        return [(self.conv1, self.bn1, 3, self.stride, 1, True), (self.conv2, self.bn2, 3, 1, 1, False)]


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample
        self.stride = stride

    def convs(self):
        return [(self.conv1, self.bn1, 1, 1, 0, True), (self.conv2, self.bn2, 3, self.stride, 1, True),
                (self.conv3, self.bn3, 1, 1, 0, False)]


class _ResNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, model):  # noqa: D401 - autograd signature
        feat, tape, lease = model._forward_train(x)
        ctx.model = model
        ctx.tape = tape
        ctx.lease = lease  # keeps a graph-owned tape marked live until backward (or until ctx is freed)
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        ctx.model._backward_impl(ctx.tape, dfeat)
        ctx.tape = None
        ctx.lease = None
        return None, None, None


class _TapeLease:
    """Marks a captured graph's static tape as holding activations a pending backward still needs.  The
    graph entry keeps only a weak reference: the lease dies when backward has consumed the tape or when the
    autograd graph that holds it is freed, and only while it is alive does a replay of the same graph fall
    back to the eager forward (which allocates a fresh tape) instead of overwriting it."""


@dataclass
class _Tape:
    stem: tuple = ()
    blocks: list = field(default_factory=list)
    out_shape: tuple = ()
    batch_stats: bool = True  # train-mode BN (batch statistics) in the forward that made the tape


class ResNetHip(nn.Module):
    def __init__(self, kind: str = "bottleneck", layers=(3, 4, 6, 3), precision: str = "bf16") -> None:
        super().__init__()
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be 'bf16' or 'fp32', got {precision!r}")
        self.precision = precision
        block = BasicBlock if kind == "basic" else Bottleneck
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        inplanes = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if i == 0 else 2
            blocks = []
            for j in range(n):
                s = stride if j == 0 else 1
                ds = None
                if j == 0 and (s != 1 or inplanes != planes * block.expansion):
                    ds = nn.Sequential(nn.Conv2d(inplanes, planes * block.expansion, 1, stride=s, bias=False),
                                       nn.BatchNorm2d(planes * block.expansion))
                blocks.append(block(inplanes, planes, s, ds))
                inplanes = planes * block.expansion
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.num_features = inplanes
        self.grad_ready_hook: Callable[[list], None] | None = None
        self._shadow: dict[int, torch.Tensor] | None = None
        # bf16 backward: the weight gradients (split-K gather GEMMs + slab finishes) of each block run on a
        # side stream beside the data-gradient / BatchNorm chain of the next one, one main->side hand-off
        # per block (SV_SIDE_STREAM=0: off, every kernel on the current stream, bitwise the same result)
        self.overlap_wgrad = os.environ.get("SV_SIDE_STREAM", "1") != "0"
        # the side stream's GEMMs run on at most 3/4 of the CUs (persistent over their tiles): a v3 wgrad
        # workgroup fills its CU's register file, so an uncapped side grid kept the dgrad / BN chain's small
        # kernels waiting for CUs (192 of 256: 3427-3438 -> 3489-3503 img/s; 128 / 160 / 224 in between)
        self.side_grid_cap: int | None = None  # None: 3/4 of the device's CUs
        self._side: dict = {}
        # training forward replayed from a captured HIP graph (per input signature; the first call runs
        # eagerly): ~250 launches of host enqueue become one, so the host stays ahead of the GPU while
        # it issues the eager backward (SV_GRAPH_FORWARD=0: eager forward, bitwise the same result)
        self.graph_forward = os.environ.get("SV_GRAPH_FORWARD", "1") != "0"
        self._fgraphs: dict = {}
        self._fwarm: set = set()
        self._fgraph_storage = None  # device storage the captured graphs read (see _storage_sig)
        self.graph_safe = True  # the whole step may be captured (StepEngine(cuda_graph=True))
        # data-parallel runs: the backward's GEMM grids (both streams) leave this many CUs to RCCL (see
        # ConvNeXtHip.comm_reserve_cus); 0 = every CU
        self.comm_reserve_cus = 0
        self.comm_cu_mask = False  # StepEngine: also mask the side stream's CUs (opt-in, see engine.py)
        self._init_weights()

    def set_weight_shadow(self, shadow: dict[int, torch.Tensor] | None) -> None:
        """Install bf16 views kept fresh by the flat optimizer (id(param) -> bf16 tensor).  A 1x1 conv
        whose channels need no padding (Cs == Cin) reads its shadow directly: [Cout][Cin][1][1] is
        already the packed [Cout][1][Cs] layout, so no per-step pack launch."""
        self._shadow = shadow
        self._drop_forward_graphs()

    def _drop_forward_graphs(self) -> None:
        self._fgraphs.clear()
        self._fwarm.clear()
        self._fgraph_storage = None

    def _storage_sig(self) -> tuple:
        """Addresses a captured forward graph has baked in: every parameter's and buffer's storage and the
        bf16 shadow views.  FlatArena (p.data rebinding), BufferSync (buffer rebinding), model.to() and a
        new shadow all change it; the graphs are then dropped and re-captured."""
        sh = self._shadow
        return (tuple(p.data_ptr() for p in self.parameters()), tuple(b.data_ptr() for b in self.buffers()),
                id(sh), tuple(t.data_ptr() for t in sh.values()) if sh else ())

    # timm ResNet.init_weights: kaiming_normal_(fan_out, relu) for convs, BN weight 1 / bias 0, and
    # zero_init_last=True: the last BN of every block starts at weight 0
    def _init_weights(self) -> None:
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for blk in self.blocks():
            nn.init.zeros_(blk.convs()[-1][1].weight)

    @property
    def compute_bf16(self) -> bool:
        return self.precision == "bf16"

    @property
    def act_dtype(self) -> torch.dtype:
        return torch.bfloat16 if self.compute_bf16 else torch.float32

    @property
    def grad_dtype(self) -> torch.dtype:
        """dtype of the backward's gradient stream (block output / input gradients)."""
        return torch.bfloat16 if self.compute_bf16 and _GRAD_BF16 else torch.float32

    def blocks(self):
        for i in range(1, 5):
            yield from getattr(self, f"layer{i}")

    # -- forward -----------------------------------------------------------------------------------
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            raise RuntimeError("ResNetHip runs on the MI355X kernel library only (got a CPU tensor)")
        # uint8 [B,H,W,3] crops (row f1, ClassificationConfig.device_transform): ToTensor + Normalize run
        # on the device inside the stem's NHWC conversion; otherwise the normalised f32 NCHW batch
        x = x.contiguous() if x.dtype == torch.uint8 else x.float().contiguous()
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if need_grad:
            anchor = torch.zeros((), device=x.device, requires_grad=True)
            return _ResNetFn.apply(x, anchor, self)
        feat, _ = self._forward_graphed(x, save=False)
        return feat

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward(x)

    def _bn(self, bn: nn.BatchNorm2d, y2d: torch.Tensor, part: torch.Tensor | None = None):
        """(mean, rstd) of a BatchNorm: batch statistics (+ running update) in train mode.  ``part``: the
        statistics partials the conv's GEMM epilogue already produced (no read pass over y)."""
        if self.training:
            momentum = 0.1 if bn.momentum is None else bn.momentum
            if part is not None:
                return K.bn_stats_from_partials(part, y2d.shape[0], eps=bn.eps, momentum=momentum,
                                                running_mean=bn.running_mean, running_var=bn.running_var,
                                                num_batches_tracked=bn.num_batches_tracked)
            mean, rstd = K.bn_stats(y2d, eps=bn.eps, momentum=momentum, running_mean=bn.running_mean,
                                    running_var=bn.running_var, num_batches_tracked=bn.num_batches_tracked)
            return mean, rstd
        return K.bn_eval_params(bn.running_mean, bn.running_var, bn.eps)

    def _small_bn(self, y4d: torch.Tensor, part: torch.Tensor | None) -> bool:
        """Train-mode BatchNorm whose statistics partials the conv produced, in a shape that K.bn_act_partials
        serves in one launch: the one-workgroup-per-8-channels form (rows <= 8192, SV_BN_SMALL) or the fold kernels
        (the fold inside the activation pass, SV_BN_FOLD)."""
        if not (self.training and part is not None and part.data_ptr() % 16 == 0):
            return False
        rows, C = y4d.numel() // y4d.shape[-1], y4d.shape[-1]
        return K.bn_small_ok(rows, C) or K.bn_fold_ok(rows, C, part.shape[0])

    @staticmethod
    def _bn_params(bn: nn.BatchNorm2d) -> tuple:
        momentum = 0.1 if bn.momentum is None else bn.momentum
        return (bn.weight.detach(), bn.bias.detach(), bn.eps, momentum, bn.running_mean, bn.running_var,
                bn.num_batches_tracked)

    def _conv(self, x4d, conv, k, stride, pad, Cin=None, packed=None):
        """conv(x) -> (y, packed weight, shape, BN-statistics partials or None); y in the activation dtype.
        In train mode (bf16) the conv GEMM's epilogue also emits the following BatchNorm's statistics.
        ``packed``: id(weight) -> its packed form from the forward's one multi-segment pack launch."""
        B, H, W, Cs = x4d.shape
        s = K.conv_shape(B, H, W, Cs, conv.weight.shape[0], k, stride, pad, Cin)
        sh = self._shadow
        if k == 1 and self.compute_bf16 and sh is not None and id(conv.weight) in sh and Cs == conv.weight.shape[1]:
            wp = sh[id(conv.weight)].view(conv.weight.shape[0], 1, Cs)
        elif packed is not None and id(conv.weight) in packed and packed[id(conv.weight)].shape[-1] == Cs:
            wp = packed[id(conv.weight)]
        else:
            wp = K.conv_weight_pack(conv.weight.detach(), Cs, self.act_dtype)
        if self.training and self.compute_bf16:
            y, part = K.conv_fwd_bn_stats(x4d, wp, s, self.act_dtype)
            return y, wp, s, part
        return K.conv_fwd(x4d, wp, s, self.act_dtype), wp, s, None

    @torch.no_grad()
    def _forward_train(self, img: torch.Tensor):
        """(features, tape, lease): the lease is None for an eager tape (a fresh allocation)."""
        return self._forward_graphed(img, save=True, leased=True)

    @torch.no_grad()
    def _forward_graphed(self, img: torch.Tensor, save: bool, leased: bool = False):
        """_forward_impl(img, save), from a captured graph when graph_forward is on: the graph owns the
        static input, the activations saved for the backward (the tape, reused by every replay) and the
        features; the caller gets a copy of the features.  BatchNorm statistics (batch or running), weight
        packing and the bf16 shadow reads all run inside the graph, so a replay is the eager forward kernel
        for kernel.  Used for the training forward and the tape-free eval / predict forward.

        A training replay whose tape a pending backward still holds (two forwards before one backward:
        a two-view loss, say) runs eagerly instead of overwriting it (``_TapeLease``)."""
        def eager():
            feat, tape = self._forward_impl(img, save=save)
            return (feat, tape, None) if leased else (feat, tape)

        if not (self.graph_forward and img.is_cuda) or torch.cuda.is_current_stream_capturing():
            return eager()  # (inside a whole-step capture: no nested graph)
        sig = self._storage_sig()
        if sig != self._fgraph_storage:  # weights / buffers / shadow rebound since the capture
            self._drop_forward_graphs()
            self._fgraph_storage = sig
        key = (tuple(img.shape), img.dtype, img.device, save, self.training)
        ent = self._fgraphs.get(key)
        if ent is None:
            if len(self._fgraphs) >= _MAX_FORWARD_GRAPHS:  # each graph keeps its activations' memory pool
                return eager()
            if key not in self._fwarm:  # first call: eager (lazy kernel attributes, caches)
                self._fwarm.add(key)
                return eager()
            static = img.clone()
            torch.cuda.synchronize(img.device)
            graph = torch.cuda.CUDAGraph()
            # thread_local: another thread's HIP calls (RCCL's proxy, a data-loader pin thread) during
            # the capture do not invalidate it
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                feat, tape = self._forward_impl(static, save=save)
            ent = self._fgraphs[key] = [static, graph, feat, tape, None]
        static, graph, feat, tape, lease_ref = ent
        if leased and lease_ref is not None and lease_ref() is not None:
            return eager()  # the static tape still belongs to a pending backward
        if static.data_ptr() != img.data_ptr():
            static.copy_(img)
        graph.replay()
        if not leased:
            return feat.clone(), tape
        lease = _TapeLease()
        ent[4] = weakref.ref(lease)
        return feat.clone(), tape, lease

    @torch.no_grad()
    def _forward_impl(self, img: torch.Tensor, save: bool):
        act = self.act_dtype
        cs0 = 8 if self.compute_bf16 else 4
        if img.dtype == torch.uint8:
            x0 = K.image_u8_hwc_to_nhwc(img, cs0, act)
        else:
            x0 = K.image_to_nhwc(img, cs0, act)
        packed = None
        if self.compute_bf16 and _MULTI_PACK:
            # every weight the convs below pack (the stem's, the 3x3s') in ONE launch instead of one each
            ws = [(self.conv1.weight, cs0)] + [(conv.weight, conv.weight.shape[1]) for blk in self.blocks()
                                               for conv, _, k, _, _, _ in blk.convs() if k > 1]
            packed = {id(w): wp for (w, _), wp in zip(ws, K.conv_weight_pack_multi(
                [(w.detach(), c) for w, c in ws], act))}
        y0, wp0, s0, p0 = self._conv(x0, self.conv1, 7, 2, 3, Cin=3, packed=packed)
        B, H, W, C = y0.shape
        if self._small_bn(y0, p0):
            a0, m0, r0 = K.bn_act_partials(y0.view(-1, C), p0, self._bn_params(self.bn1), relu=True, out_dtype=act)
        else:
            m0, r0 = self._bn(self.bn1, y0.view(-1, C), p0)
            a0 = K.bn_act(y0.view(-1, C), m0, r0, self.bn1.weight, self.bn1.bias, relu=True, out_dtype=act)
        a0 = a0.view(B, H, W, C)
        x, idx = K.maxpool_fwd(a0)
        tape = _Tape(batch_stats=self.training) if save else None
        if save:
            tape.stem = (x0, y0, m0, r0, a0, idx, wp0, s0)
        for blk in self.blocks():
            x_in = x
            cur = x
            saved = []
            convs = blk.convs()
            last_part = None  # the last BatchNorm's partials when its statistics join the residual launch
            for ci, (conv, bn, k, st, pad, relu) in enumerate(convs):
                y, wp, s, part = self._conv(cur, conv, k, st, pad, packed=packed)
                Bq, Hq, Wq, Cq = y.shape
                last = ci == len(convs) - 1
                small = self._small_bn(y, part)
                if not last:
                    if small:  # statistics fold + BatchNorm + ReLU in one launch (bit for bit the two below)
                        a, mean, rstd = K.bn_act_partials(y.view(-1, Cq), part, self._bn_params(bn), relu=True,
                                                       out_dtype=act)
                    else:
                        mean, rstd = self._bn(bn, y.view(-1, Cq), part)
                        a = K.bn_act(y.view(-1, Cq), mean, rstd, bn.weight, bn.bias, relu=True, out_dtype=act)
                    a = a.view(Bq, Hq, Wq, Cq)
                    saved.append((cur, y, mean, rstd, a, wp, s))
                    cur = a
                elif small:
                    last_part = part
                    saved.append((cur, y, None, None, None, wp, s))
                else:
                    mean, rstd = self._bn(bn, y.view(-1, Cq), part)
                    saved.append((cur, y, mean, rstd, None, wp, s))
            # residual join: out = relu(bn_last(y) + shortcut), shortcut = x or BN(conv_ds(x))
            c_last, y_last, m_last, r_last, _, wp_last, s_last = saved[-1]
            bn_last = convs[-1][1]
            Bq, Hq, Wq, Cq = y_last.shape
            ds_saved = None
            if blk.downsample is not None:
                dconv, dbn = blk.downsample[0], blk.downsample[1]
                yd, wpd, sd, pd = self._conv(x_in, dconv, 1, blk.stride, 0)
                if last_part is not None and self._small_bn(yd, pd):
                    out, m_last, r_last, md, rd = K.bn_act_partials(
                        y_last.view(-1, Cq), last_part, self._bn_params(bn_last), res=yd.view(-1, Cq), res_part=pd,
                        res_params=self._bn_params(dbn), relu=True, out_dtype=act)
                else:
                    if last_part is not None:
                        m_last, r_last = self._bn(bn_last, y_last.view(-1, Cq), last_part)
                    md, rd = self._bn(dbn, yd.view(-1, Cq), pd)
                    out = K.bn_act(y_last.view(-1, Cq), m_last, r_last, bn_last.weight, bn_last.bias,
                                   res=yd.view(-1, Cq), res_bn=(md, rd, dbn.weight, dbn.bias), relu=True, out_dtype=act)
                ds_saved = (yd, md, rd, wpd, sd)
            elif last_part is not None:
                out, m_last, r_last = K.bn_act_partials(y_last.view(-1, Cq), last_part, self._bn_params(bn_last),
                                                     res=x_in.view(-1, Cq), relu=True, out_dtype=act)
            else:
                out = K.bn_act(y_last.view(-1, Cq), m_last, r_last, bn_last.weight, bn_last.bias,
                               res=x_in.view(-1, Cq), relu=True, out_dtype=act)
            saved[-1] = (c_last, y_last, m_last, r_last, None, wp_last, s_last)
            out = out.view(Bq, Hq, Wq, Cq)
            if save:
                tape.blocks.append((x_in, saved, ds_saved, out))
            x = out
        feat = K.avgpool_fwd(x)
        if save:
            tape.out_shape = tuple(x.shape)
        return feat, tape

    # -- backward ----------------------------------------------------------------------------------
    @staticmethod
    def _grad(p: torch.Tensor) -> torch.Tensor:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        return p.grad

    def _ready(self, params: list) -> None:
        if self.grad_ready_hook is not None:
            self.grad_ready_hook(params)

    def _side_stream(self, device) -> torch.cuda.Stream:
        """The weight-gradient side stream; CU-masked (never on the CUs reserved for RCCL, training/cumask.py) when
        StepEngine asks for it (comm_reserve_cus > 0 and SV_COMM_CU_MASK=1)."""
        key = (device, self.comm_reserve_cus, self.comm_cu_mask)
        if key not in self._side:
            if self.comm_reserve_cus > 0 and self.comm_cu_mask:
                from ..training.cumask import reserved_stream

                self._side[key] = reserved_stream(device, self.comm_reserve_cus, "side")
            else:
                self._side[key] = torch.cuda.Stream(device=device)
        return self._side[key]

    def _flush_wgrads(self, jobs: list, params: list, side, keep: list, deferred: list | None = None,
                      pol: "nv.GemmPolicy | None" = None) -> None:
        """Run the block's weight gradients (conv_bwd_weight jobs) and report its parameters ready.  With a
        side stream: one hand-off (the side stream waits for everything the main stream has issued, so the
        grad-ready event it records also covers the BatchNorm gradients), and the operands stay referenced
        in ``keep`` until the streams join (the main stream's allocator may not reuse them earlier)."""
        if side is None:
            for dy4, x, s, dw in jobs:
                K.conv_bwd_weight(dy4, x, s, dw=dw, accumulate=True, policy=pol)
            if deferred is not None:  # reported after the streams join (a bucket may hold side-stream grads)
                deferred.extend(params)
            else:
                self._ready(params)
            return
        side.wait_event(torch.cuda.current_stream().record_event())
        ncu = torch.cuda.get_device_properties(side.device).multi_processor_count
        if self.side_grid_cap is None:
            self.side_grid_cap = ncu * 3 // 4
        cap = self.side_grid_cap
        if self.comm_reserve_cus > 0:
            cap = min(cap, max(1, ncu - self.comm_reserve_cus))
        spol = nv.policy(grid_cap=cap)  # the side stream's own policy, passed with each call
        with torch.cuda.stream(side):
            for dy4, x, s, dw in jobs:
                K.conv_bwd_weight(dy4, x, s, dw=dw, accumulate=True, policy=spol)
            self._ready(params)
        keep.append(jobs)

    @torch.no_grad()
    def _block_backward(self, blk, saved_block, d: torch.Tensor, side=None, keep=None, deferred=None,
                        batch_stats: bool = True, pol: "nv.GemmPolicy | None" = None,
                        pending: list | None = None) -> torch.Tensor:
        """Backward of one residual block given d = dL/d(block output) (``grad_dtype``, NHWC, contiguous);
        accumulates the block's parameter gradients and returns dL/d(block input) (``grad_dtype``).

        ``d`` is CLOBBERED: the block-output BatchNorm's statistics pass writes the ReLU-masked gradient over it
        (it is the shortcut's gradient), and an identity block returns that same buffer with the main path's data
        gradient added.  Callers pass a buffer they own (the next block's dx, or the pooling gradient)."""
        assert d.is_contiguous() and d.dtype == self.grad_dtype, \
            "_block_backward: d must be a contiguous grad_dtype buffer the caller owns (it is overwritten)"
        act = self.act_dtype
        g = self._grad
        jobs = []
        x_in, saved, ds_saved, out = saved_block
        convs = blk.convs()
        Bq, Hq, Wq, Cq = out.shape
        rows = Bq * Hq * Wq
        # last BN of the main path, with the block-output ReLU mask; gm = the masked gradient, written over
        # d by the statistics pass (d is this block's own: the next block's dx or the pooling gradient)
        gm = d.reshape(rows, Cq)
        conv, bn, _, _, _, _ = convs[-1]
        cur_in, y, mean, rstd, _, wp, s = saved[-1]
        dyd = None
        if ds_saved is not None and _BN_DUAL:
            # the shortcut's BatchNorm from the same masked gradient, in the same two passes (gm read once)
            yd, md, rd, _, _ = ds_saved
            dbn = blk.downsample[1]
            dy, dyd = K.bn_bwd_dual(gm, y.view(rows, Cq), mean, rstd, bn.weight, out.view(rows, Cq),
                                    yd.view(rows, Cq), md, rd, dbn.weight, dgamma=g(bn.weight), dbeta=g(bn.bias),
                                    dgamma2=g(dbn.weight), dbeta2=g(dbn.bias), dx_dtype=act,
                                    batch_stats=batch_stats)
        else:
            dy = K.bn_bwd(gm, y.view(rows, Cq), mean, rstd, bn.weight, act=out.view(rows, Cq),
                          dgamma=g(bn.weight), dbeta=g(bn.bias), dx_dtype=act, mask_inplace=True,
                          batch_stats=batch_stats)
        self._flush_pending(pending)  # the previous block's weight gradients, now that the main queue has work
        params = [bn.weight, bn.bias]
        for ci in range(len(convs) - 1, -1, -1):
            conv, bn, _, _, _, _ = convs[ci]
            cur_in, y, mean, rstd, a, wp, s = saved[ci]
            dy4 = dy.view(y.shape)
            jobs.append((dy4, cur_in, s, g(conv.weight)))
            params.append(conv.weight)
            if ci == 0:
                break
            pconv, pbn, _, _, _, _ = convs[ci - 1]
            _, py, pmean, prstd, pa, _, _ = saved[ci - 1]
            Cp = py.shape[-1]
            # the inner BN's backward statistics from the data gradient's GEMM epilogue / split-K finish where
            # that path carries them (bf16; stride 2 on even grids without a split), else from bn_bwd's own
            # statistics pass
            fused = (K.conv_bwd_data_bn(dy4, wp, s, py, pmean, prstd, pbn.weight, pbn.bias,
                                        unsplit=_BN_BWD_EPI != "split" or (s.stride == 2 and _S2_BN),
                                        policy=pol)
                     if _BN_BWD_EPI != "0" and act == torch.bfloat16 else None)
            da, bpart = fused if fused is not None else (K.conv_bwd_data(dy4, wp, s, dx_dtype=act, policy=pol), None)
            # the inner BN's own ReLU: mask recomputed from y (the activation pa is not read again)
            dy = K.bn_bwd(da.view(-1, Cp), py.view(-1, Cp), pmean, prstd, pbn.weight, relu_beta=pbn.bias.detach(),
                          dgamma=g(pbn.weight), dbeta=g(pbn.bias), dx_dtype=act,
                          batch_stats=batch_stats, part=bpart)
            params += [pbn.weight, pbn.bias]
        # dy is now the gradient at conv1's output; conv1's input is x_in
        s1, wp1 = saved[0][6], saved[0][5]
        if ds_saved is not None:
            yd, md, rd, wpd, sd = ds_saved
            dconv, dbn = blk.downsample[0], blk.downsample[1]
            if dyd is None:
                dyd = K.bn_bwd(gm, yd.view(rows, Cq), md, rd, dbn.weight, dgamma=g(dbn.weight), dbeta=g(dbn.bias),
                               dx_dtype=act, batch_stats=batch_stats)
            dyd4 = dyd.view(yd.shape)
            jobs.append((dyd4, x_in, sd, g(dconv.weight)))
            # conv1's data gradient first (a plain store), then the strided shortcut's added onto the
            # one output parity class its 1x1 taps reach (the other three are skipped, not rewritten)
            dx = K.conv_bwd_data(dy.view(saved[0][1].shape), wp1, s1, dx_dtype=self.grad_dtype, policy=pol)
            K.conv_bwd_data(dyd4, wpd, sd, dx=dx, accumulate=True, policy=pol)
            params += [dconv.weight, dbn.weight, dbn.bias]
        else:
            dx = gm.view(x_in.shape)  # identity shortcut: the masked gradient flows straight through
            K.conv_bwd_data(dy.view(saved[0][1].shape), wp1, s1, dx=dx, accumulate=True, policy=pol)
        if pending is not None and side is not None:
            pending.append((jobs, params, side, keep, deferred, pol))
        else:
            self._flush_wgrads(jobs, params, side, keep, deferred, pol)
        return dx

    def _flush_pending(self, pending: list | None) -> None:
        while pending:
            self._flush_wgrads(*pending.pop(0))

    @torch.no_grad()
    def _backward_impl(self, tape: _Tape, dfeat: torch.Tensor) -> None:
        act = self.act_dtype
        g = self._grad
        main = torch.cuda.current_stream()
        side = self._side_stream(main.device) if (self.overlap_wgrad and self.compute_bf16) else None
        main_cap = 0
        if self.comm_reserve_cus > 0:
            main_cap = max(1, torch.cuda.get_device_properties(main.device).multi_processor_count - self.comm_reserve_cus)
        pol = nv.policy(grid_cap=main_cap)  # the main stream's GEMM policy, passed with each call
        keep: list = []
        deferred: list | None = [] if side is not None else None
        pending: list | None = [] if (_DEFER_FLUSH and side is not None) else None
        d = K.avgpool_bwd(dfeat, tape.out_shape, dx_dtype=self.grad_dtype)  # gradient of the last block output
        blocks = list(self.blocks())
        for i, (blk, saved_block) in zip(range(len(blocks) - 1, -1, -1), zip(reversed(blocks), reversed(tape.blocks))):
            # every block's weight gradients on the side stream: the first block's run beside the main
            # stream's tail (its data gradients, the max-pool / stem BatchNorm backward and the stem's
            # weight gradient, which stays on the main stream as the last producer); the side queue is
            # empty by then (r4k trace), so they no longer wait behind a backlog: +0.5 % (r4s A/B)
            d = self._block_backward(blk, saved_block, d, side if (i > 0 or _FIRST_BLOCK_SIDE) else None, keep,
                                     deferred, batch_stats=tape.batch_stats, pol=pol, pending=pending)
        # stem: maxpool -> BN + ReLU -> conv7x7 (weight gradient only)
        x0, y0, m0, r0, a0, idx, wp0, s0 = tape.stem
        B, H, W, C = a0.shape
        if _POOLED_STEM_BWD:  # the max-pool backward gathered inside the stem BN's two passes
            dy0 = K.bn_relu_bwd_pooled(d, idx, H, W, y0.view(-1, C), m0, r0, self.bn1.weight, self.bn1.bias.detach(),
                                       dgamma=g(self.bn1.weight), dbeta=g(self.bn1.bias), dx_dtype=act,
                                       batch_stats=tape.batch_stats)
        else:
            da0 = K.maxpool_bwd(d, idx, H, W, dx_dtype=torch.float32)
            dy0 = K.bn_bwd(da0.view(-1, C), y0.view(-1, C), m0, r0, self.bn1.weight, relu_beta=self.bn1.bias.detach(),
                           dgamma=g(self.bn1.weight), dbeta=g(self.bn1.bias), dx_dtype=act,
                           batch_stats=tape.batch_stats)
        self._flush_pending(pending)
        self._flush_wgrads([(dy0.view(y0.shape), x0, s0, g(self.conv1.weight))],
                           [self.conv1.weight, self.bn1.weight, self.bn1.bias], None, keep, deferred, pol)
        if side is not None:
            main.wait_stream(side)  # clip / AdamW / the next step see every side-stream gradient
            self._ready(deferred)
        keep.clear()


def create_resnet(name: str, precision: str = "bf16") -> ResNetHip:
    key = name.split(".")[0]
    if key not in RESNET_CFGS:
        raise ValueError(f"unsupported ResNet variant {name!r}")
    kind, layers = RESNET_CFGS[key]
    return ResNetHip(kind, layers, precision=precision)
