"""ConvNeXt backbone on the gfx950 kernel library -- drop-in for
``timm.create_model("convnext_{base,large}...", num_classes=0)`` as called at
spine_vision/training/models/backbone.py:166-170 (timm 1.0.22 ``timm/models/convnext.py``).

* Same module tree and ``state_dict`` keys as timm (``stem.{0,1}``, ``stages.i.downsample.{0,1}``,
  ``stages.i.blocks.j.{conv_dw,norm,mlp.fc1,mlp.fc2,gamma}``, ``head.norm``), ``num_features``,
  ``forward([B,3,H,W] f32) -> [B,F]``.  The sub-modules are parameter containers only; their own
  ``forward`` is never called.
* Forward and backward are explicit sequences of HIP kernels over NHWC activations (see
  DESIGN.md "ConvNeXt step"): stem conv+LN, per block {dwconv7 -> LN, fc1 GEMM (+bias, +GELU),
  fc2 GEMM (+bias, *gamma, +residual)}, downsample LN+patch GEMM, pool+LN.  Backward writes the
  parameter gradients straight into ``p.grad`` (views of the trainer's flat gradient buffer) and
  calls ``grad_ready_hook`` after each block so the DDP bucketer can start its all-reduce while the
  remaining blocks are still being differentiated.
* ``precision="bf16"``: bf16 MFMA, bf16 saved activations, f32 residual/gradient streams, f32
  master weights.  ``precision="fp32"``: every tensor f32 and f32 MFMA (parity mode, <=1e-3 vs the
  reference CPU path).
"""

from __future__ import annotations

import os
from contextlib import nullcontext as _nullctx
from dataclasses import dataclass, field
from typing import Callable

import torch
import torch.nn as nn

from .. import kernels as K
from .. import native as nv

CONVNEXT_CFGS = {
    "convnext_tiny": ((3, 3, 9, 3), (96, 192, 384, 768)),
    "convnext_small": ((3, 3, 27, 3), (96, 192, 384, 768)),
    "convnext_base": ((3, 3, 27, 3), (128, 256, 512, 1024)),
    "convnext_large": ((3, 3, 27, 3), (192, 384, 768, 1536)),
}


def _comm_cap(device, reserve: int) -> int:
    """GEMM grid cap that leaves ``reserve`` CUs to the comm stream (0: no cap)."""
    if reserve <= 0:
        return 0
    return max(1, torch.cuda.get_device_properties(device).multi_processor_count - reserve)


class _Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int) -> None:
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class ConvNeXtBlock(nn.Module):
    """Parameter container for timm ConvNeXtBlock (conv_mlp=False, ls_init_value, no drop_path)."""

    def __init__(self, dim: int, ls_init_value: float = 1e-6) -> None:
        super().__init__()
        self.conv_dw = nn.Conv2d(dim, dim, kernel_size=7, padding=3, groups=dim, bias=True)
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _Mlp(dim, 4 * dim)
        self.gamma = nn.Parameter(ls_init_value * torch.ones(dim))


class ConvNeXtStage(nn.Module):
    def __init__(self, in_chs: int, out_chs: int, depth: int, downsample: bool) -> None:
        super().__init__()
        if downsample:
            self.downsample = nn.Sequential(nn.LayerNorm(in_chs, eps=1e-6), nn.Conv2d(in_chs, out_chs, 2, stride=2))
        else:
            self.downsample = nn.Identity()
        self.blocks = nn.Sequential(*[ConvNeXtBlock(out_chs) for _ in range(depth)])


class _Head(nn.Module):
    def __init__(self, dim: int) -> None:
        super().__init__()
        self.norm = nn.LayerNorm(dim, eps=1e-6)


@dataclass
class _Tape:
    """Activations saved by the training forward for the explicit backward."""

    img: torch.Tensor
    stem: tuple = ()
    stages: list = field(default_factory=list)  # per stage: (ds_saved or None, [block_saved...])
    pool: tuple = ()
    out_shape: tuple = ()
    wcache: dict = field(default_factory=dict)  # bf16 weight casts shared by forward and backward
    w2g: dict = field(default_factory=dict)  # bf16 (fc2 weight x gamma) per block, for the fc2 dgrad
    wt: dict = field(default_factory=dict)  # (bf16 (W2 gamma)^T, bf16 W1^T) per block of the fused MLP backward
    w2g_ready: object = None  # event on the side stream after the last w2g


class _ConvNeXtFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, model):  # noqa: D401 - autograd signature
        feat, tape = model._forward_impl(x, save=True)
        ctx.model = model
        ctx.tape = tape
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        ctx.model._backward_impl(ctx.tape, dfeat)
        ctx.tape = None
        return None, None, None


# the backward's last block: its fc1 and depthwise weight gradients on the main stream after the stem, not behind the
# side stream's backlog.  Opt-in (SV_TAIL_MAIN=1): the step's end waited ~0.5 ms on the side stream (r11k trace), but
# moving them measured no different (1088.7-1092.2 vs 1090.7-1091.2 img/s interleaved, r11m); neither did letting the
# lean release keep 64 blocks of side-stream operands instead of 4 (SV_RELEASE_BATCH: 1092.7-1092.8)
# SV_TAIL_MAIN=2: the same jobs on the main stream BEFORE the stem's backward (the side stream then ends with the block's
# fc2 weight gradient while the main stream runs them and the stem): 1115.3-1120.6 vs 1116.6-1119.0 img/s (r11s)
_TAIL_MAIN = int(os.environ.get("SV_TAIL_MAIN", "0"))


class ConvNeXtHip(nn.Module):
    def __init__(self, depths=(3, 3, 27, 3), dims=(128, 256, 512, 1024), ls_init_value: float = 1e-6,
                 precision: str = "bf16") -> None:
        super().__init__()
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be 'bf16' or 'fp32', got {precision!r}")
        self.depths, self.dims = tuple(depths), tuple(dims)
        self.precision = precision
        self.stem = nn.Sequential(nn.Conv2d(3, dims[0], kernel_size=4, stride=4), nn.LayerNorm(dims[0], eps=1e-6))
        stages = []
        prev = dims[0]
        for i, (d, c) in enumerate(zip(depths, dims)):
            stages.append(ConvNeXtStage(prev, c, d, downsample=i > 0))
            prev = c
        self.stages = nn.Sequential(*stages)
        self.norm_pre = nn.Identity()
        self.head = _Head(prev)
        self.num_features = self.head_hidden_size = prev
        self.grad_ready_hook: Callable[[list], None] | None = None
        self._shadow: dict[int, torch.Tensor] | None = None  # id(param) -> bf16 shadow view
        # weight-gradient kernels on a side stream beside the data-gradient chain (SV_SIDE_STREAM=0: off)
        self.overlap_wgrad = os.environ.get("SV_SIDE_STREAM", "1") != "0"
        self.side_wg_per_cu = 1  # the data-gradient GEMMs keep one workgroup per CU free for the side stream
        # bf16 backward: ONE main->side hand-off per block (after the LayerNorm backward) instead of three,
        # and the side stream's operands kept alive in a list until the streams join instead of
        # record_stream -- every cross-stream event / allocator event is a release packet (L2 write-back)
        self.lean_sync = os.environ.get("SV_LEAN_SYNC", "1") != "0"
        self._side: dict = {}
        # the lean backward polls side-stream events (_release_side), which a stream capture forbids:
        # StepEngine(cuda_graph=True) refuses this backbone
        self.graph_safe = False
        # data-parallel runs (StepEngine, world > 1): the backward's persistent GEMM grids leave this many
        # CUs free so RCCL's all-reduce kernels on the comm stream find a CU (a v9 workgroup holds its CU's
        # LDS for the whole launch); 0 = every CU
        self.comm_reserve_cus = 0
        self.comm_cu_mask = False  # StepEngine: also mask the side stream's CUs (opt-in, see engine.py)
        # a block's fc1 wgrad slab / bias, LayerNorm and depthwise partials folded by ONE launch
        # (sv_reduce_partials_multi) instead of four (SV_MERGED_FOLDS=0: one launch per fold, A/B only)
        self.merge_folds = os.environ.get("SV_MERGED_FOLDS", "1") != "0"
        # the lean side stream's GEMMs on at most this many workgroups (None: every CU; SV_SIDE_GRID_CAP)
        cap = os.environ.get("SV_SIDE_GRID_CAP")
        self.side_grid_cap: int | None = int(cap) if cap else None
        # the side stream's weight-gradient GEMM family (sv_gemm_policy.impl; 0 = the measured dispatch, A/B runs)
        self.side_impl = int(os.environ.get("SV_WGRAD_IMPL", "0"))
        # a grid cap on the main stream's backward GEMMs (A/B runs; 128 measured equal to none, 192/224 slower:
        # profiles/round4/r9u_main_cap_and_tile_queue_rejected.txt)
        self.main_bwd_cap = int(os.environ.get("SV_MAIN_BWD_CAP", "0"))
        # the block weight gradients' persistent grid target (kernels._wgrad_split_for): with bf16 split-K slabs the
        # whole chip (256) beats half of it (128) here, +0.8 % (1108-1112 vs 1097-1105 img/s interleaved; ResNet's
        # stay at 128, where 256 measured -2 %: profiles/round4/r9zn_wgrad_target_bf16_slabs.txt); SV_CNX_WGRAD_WGS
        self.wgrad_target = int(os.environ.get("SV_CNX_WGRAD_WGS", "256"))
        # the side stream's GEMMs at raised wave priority (SV_SIDE_PRIO=0: normal, A/B runs)
        self.side_prio = int(os.environ.get("SV_SIDE_PRIO", "1"))
        # bf16 blocks of the narrow stages (C in kernels.MLP_FUSED_C) run fc1 -> GELU -> fc2 -> gamma -> + x as ONE
        # kernel (sv_mlp_fwd): the hidden activation never makes the HBM round trip between the two GEMMs; bit for
        # bit the two-GEMM path (SV_FUSED_MLP=0, A/B runs)
        self.fused_mlp = os.environ.get("SV_FUSED_MLP", "1") != "0"
        # the fused-MLP channel widths in use: S1 / S2 (and -large S1); the C = 512 kernel (S3) measured slower than the
        # two GEMMs and stays opt-in (SV_FUSED_MLP_C=128,192,256,512; csrc/mlp.hip c512)
        self.fused_mlp_c = tuple(int(c) for c in os.environ.get("SV_FUSED_MLP_C", "128,192,256").split(",") if c)
        # ... and its backward (C in kernels.MLP_BWD_FUSED_C, the bf16 lean side-stream backward): the fc2 data gradient
        # (x GELU'), the fc1 data gradient and the LayerNorm backward as ONE kernel (sv_mlp_bwd): dh is not read back and
        # dy never reaches HBM (SV_FUSED_MLP_BWD=0: the three kernels, A/B runs)
        self.fused_mlp_bwd = os.environ.get("SV_FUSED_MLP_BWD", "1") != "0"
        # StepEngine(overlap_optimizer=True) installs a training.engine.ParamGate: the forward then waits for each
        # stage's chunk of the previous step's AdamW just before the stage instead of for the whole update
        self.param_gate = None
        self._init_weights()

    def param_gate_groups(self) -> list[nn.Module]:
        """The parameter groups in forward (and arena) order, one optimizer chunk each (training.engine.ParamGate)."""
        return [self.stem, *self.stages, self.head]

    # -- timm-style init (ConvNeXt._init_weights): trunc_normal(.02) for conv/linear, zero bias
    def _init_weights(self) -> None:
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    # -- precision / weight shadows --------------------------------------------------------------
    @property
    def compute_bf16(self) -> bool:
        return self.precision == "bf16"

    @property
    def act_dtype(self) -> torch.dtype:
        return torch.bfloat16 if self.compute_bf16 else torch.float32

    def set_weight_shadow(self, shadow: dict[int, torch.Tensor] | None) -> None:
        """Install bf16 views kept fresh by the flat optimizer (id(param) -> bf16 tensor)."""
        self._shadow = shadow

    def gemm_weight_params(self) -> list[nn.Parameter]:
        ps = [self.stem[0].weight]
        for st in self.stages:
            if not isinstance(st.downsample, nn.Identity):
                ps.append(st.downsample[1].weight)
            for blk in st.blocks:
                ps += [blk.mlp.fc1.weight, blk.mlp.fc2.weight]
        return ps

    def _w(self, p: torch.Tensor, cache: dict) -> torch.Tensor:
        """Weight as the GEMM reads it: f32 param (fp32 mode) or its bf16 shadow."""
        if not self.compute_bf16:
            return p.detach()
        if self._shadow is not None and id(p) in self._shadow:
            return self._shadow[id(p)]
        k = id(p)
        if k not in cache:
            cache[k] = K.cast_bf16(p.detach().contiguous())
        return cache[k]

    # -- forward -----------------------------------------------------------------------------------
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            raise RuntimeError("ConvNeXtHip runs on the MI355X kernel library only (got a CPU tensor)")
        if x.dtype == torch.uint8:
            # decoded grayscale batch [B,H,W] (row f1): the reference transform runs on the device --
            # inside the stem gather (bf16) or as the standalone normalise kernel (fp32 parity mode)
            x = x.contiguous() if self.compute_bf16 else K.normalize_u8_gray(x.contiguous())
        else:
            x = x.float().contiguous()
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if need_grad:
            anchor = torch.zeros((), device=x.device, requires_grad=True)
            return _ConvNeXtFn.apply(x, anchor, self)
        feat, _ = self._forward_impl(x, save=False)
        return feat

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward(x)

    @torch.no_grad()
    def _forward_impl(self, img: torch.Tensor, save: bool):
        bf = self.compute_bf16
        act = self.act_dtype
        tape = _Tape(img=img) if save else None
        cache: dict = tape.wcache if save else {}
        stem_conv, stem_ln = self.stem[0], self.stem[1]
        gate = self.param_gate
        if gate is not None:
            gate.wait(self.stem)
        if save and bf and self.overlap_wgrad:
            # the fc2 dgrad operand bf16(W2 * gamma) of every block, made on the (otherwise idle during
            # the forward) side stream beside the forward; the backward waits on one event
            # (allocated on the main stream, which frees them after waiting on w2g_ready: no
            # record_stream, whose allocator event is one more release packet per tensor)
            main = torch.cuda.current_stream()
            side = self._side_stream(main.device)
            blocks = [blk for st in self.stages for blk in st.blocks]
            fused_b = {id(blk) for blk in blocks if self._fused_bwd(blk)}
            for blk in blocks:
                if id(blk) in fused_b:
                    w1, w2 = blk.mlp.fc1.weight, blk.mlp.fc2.weight
                    tape.wt[id(blk)] = (torch.empty(w2.shape[1], w2.shape[0], device=img.device, dtype=torch.bfloat16),
                                        torch.empty(w1.shape[1], w1.shape[0], device=img.device, dtype=torch.bfloat16))
                else:
                    tape.w2g[id(blk)] = torch.empty(blk.mlp.fc2.weight.shape, device=img.device, dtype=torch.bfloat16)
            side.wait_event(main.record_event())
            if gate is not None:  # every block's weights: the whole update
                gate.wait_all(side)
            with torch.cuda.stream(side):
                for blk in blocks:
                    if id(blk) in fused_b:
                        w2t, w1t = tape.wt[id(blk)]
                        K.transpose_scale_bf16(blk.mlp.fc2.weight.detach(), blk.gamma.detach(), out=w2t)
                        K.transpose_scale_bf16(blk.mlp.fc1.weight.detach(), None, out=w1t)
                    else:
                        K.scale_rows_bf16(blk.mlp.fc2.weight.detach(), blk.gamma.detach(), out=tape.w2g[id(blk)])
            tape.w2g_ready = side.record_event()
        if bf:
            # stem conv on MFMA: 4x4 patch rows (bf16, K padded to 64) x packed weight, then LayerNorm2d
            B, H0, W0 = img.shape[0], img.shape[-2], img.shape[-1]
            C0 = stem_conv.weight.shape[0]
            patches = K.stem_patchify(img)
            z0 = torch.empty(patches.shape[0], C0, device=img.device, dtype=act)
            K.linear_fwd(patches, K.stem_weight_pack(stem_conv.weight.detach()), out=z0, bias=stem_conv.bias,
                         compute_bf16=True)
            x2d, s_mean, s_rstd = K.layernorm_fwd(z0, stem_ln.weight, stem_ln.bias, out_dtype=torch.float32)
            x = x2d.view(B, H0 // 4, W0 // 4, C0)
            if save:
                tape.stem = (patches, z0, s_mean, s_rstd)
        else:
            x, s_mean, s_rstd = K.stem_fwd(img, stem_conv.weight, stem_conv.bias, stem_ln.weight, stem_ln.bias)
            if save:
                tape.stem = (s_mean, s_rstd)
        for st in self.stages:
            if gate is not None:
                gate.wait(st)
            ds_saved = None
            if not isinstance(st.downsample, nn.Identity):
                ln, conv = st.downsample[0], st.downsample[1]
                B, H, W, C = x.shape
                patches, d_mean, d_rstd = K.downsample_fwd(x, ln.weight, ln.bias, act_dtype=act)
                Cout = conv.weight.shape[0]
                wds = self._w(conv.weight, cache).reshape(Cout, 4 * C)
                xn = torch.empty(B, H // 2, W // 2, Cout, device=x.device, dtype=torch.float32)
                K.linear_fwd(patches, wds, out=xn.view(-1, Cout), bias=conv.bias, compute_bf16=bf)
                if save:
                    ds_saved = (x, patches, d_mean, d_rstd)
                x = xn
            blocks_saved = []
            for blk in st.blocks:
                B, H, W, C = x.shape
                M = B * H * W
                # the tape-free forward keeps no conv output (the one-pass depthwise + LayerNorm then writes none)
                z, y, mean, rstd = K.dwconv7_ln_fwd(x, blk.conv_dw.weight, blk.conv_dw.bias, blk.norm.weight,
                                                    blk.norm.bias, act_dtype=act, save_z=save)
                w1 = self._w(blk.mlp.fc1.weight, cache)
                w2 = self._w(blk.mlp.fc2.weight, cache)
                if bf and self.fused_mlp and C in K.MLP_FUSED_C and C in self.fused_mlp_c:
                    # fused MLP: the training forward stores GELU'(h) and GELU(h) for the backward, the eval one nothing
                    xo = torch.empty(B, H, W, C, device=x.device, dtype=torch.float32)
                    gh = torch.empty(M, 4 * C, device=x.device, dtype=act) if save else None
                    a = torch.empty(M, 4 * C, device=x.device, dtype=act) if save else None
                    K.mlp_fwd(y, w1, blk.mlp.fc1.bias, w2, blk.mlp.fc2.bias, blk.gamma, x.view(M, C), out=xo.view(M, C),
                              gelu_grad=gh, gelu_out=a)
                    if save:
                        blocks_saved.append((x, z, y, mean, rstd, gh, a))
                    x = xo
                    continue
                # fc1 epilogue: a = GELU(h) (fc2 operand) and gh = GELU'(h) (for the backward), one erf;
                # the tape-free forward (eval / predict) writes a only
                a = torch.empty(M, 4 * C, device=x.device, dtype=act)
                if save:
                    gh = torch.empty(M, 4 * C, device=x.device, dtype=act)
                    K.linear_fwd(y, w1, out=gh, out2=a, bias=blk.mlp.fc1.bias, epilogue=nv.SV_EPI_BIAS_GELU_DUAL,
                                 compute_bf16=bf)
                else:
                    gh = None
                    K.linear_fwd(y, w1, out=a, bias=blk.mlp.fc1.bias, epilogue=nv.SV_EPI_BIAS_GELU,
                                 compute_bf16=bf)
                xo = torch.empty(B, H, W, C, device=x.device, dtype=torch.float32)
                K.linear_fwd(a, w2, out=xo.view(M, C), bias=blk.mlp.fc2.bias, gamma=blk.gamma,
                             residual=x.view(M, C), epilogue=nv.SV_EPI_BIAS_GAMMA_RES, compute_bf16=bf)
                if save:
                    blocks_saved.append((x, z, y, mean, rstd, gh, a))
                x = xo
            if save:
                tape.stages.append((ds_saved, blocks_saved))
        if gate is not None:  # the head norm here, the model's heads after the return
            gate.wait_all()
        feat, pooled, p_mean, p_rstd = K.pool_ln_fwd(x, self.head.norm.weight, self.head.norm.bias)
        if save:
            tape.pool = (pooled, p_mean, p_rstd)
            tape.out_shape = tuple(x.shape)
            if tape.w2g_ready is not None:
                # the main stream owns the w2g buffers: join the side stream's writes before any path
                # (backward, or a tape dropped without one) can free them (long finished by now)
                torch.cuda.current_stream().wait_event(tape.w2g_ready)
                tape.w2g_ready = None
        return feat, tape

    # -- backward ----------------------------------------------------------------------------------
    def _fused_bwd(self, blk) -> bool:
        """Whether this block's backward runs the fused fc2 -> fc1 -> LayerNorm data-gradient kernel (bf16 lean
        side-stream schedule only: its operand images are made beside the forward)."""
        return (self.fused_mlp_bwd and self.compute_bf16 and self.overlap_wgrad and self.lean_sync
                and blk.conv_dw.weight.shape[0] in K.MLP_BWD_FUSED_C)

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

    @staticmethod
    def _grad(p: torch.Tensor) -> torch.Tensor:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        return p.grad

    def _ready(self, params: list) -> None:
        if self.grad_ready_hook is not None:
            self.grad_ready_hook(params)

    @torch.no_grad()
    def _backward_impl(self, tape: _Tape, dfeat: torch.Tensor) -> None:
        bf = self.compute_bf16
        act = self.act_dtype
        cache: dict = tape.wcache
        g = self._grad
        hn = self.head.norm
        main = torch.cuda.current_stream()
        side = self._side_stream(main.device) if self.overlap_wgrad else None
        # the backward's GEMM launch policy, passed with every call (no process-wide state): block GEMMs of
        # the two streams on one persistent workgroup per CU each, so they share every CU; under data
        # parallelism every grid leaves comm_reserve_cus CUs to RCCL
        comm_cap = _comm_cap(main.device, self.comm_reserve_cus)
        if self.main_bwd_cap > 0:
            comm_cap = min(comm_cap, self.main_bwd_cap) if comm_cap > 0 else self.main_bwd_cap
        pol = nv.policy(grid_cap=comm_cap, wg_per_cu=self.side_wg_per_cu if side is not None else 0)
        lean = side is not None and bf and self.lean_sync
        tail: list = []  # the last block's weight gradients the main stream runs after the stem (_TAIL_MAIN)
        # lean mode: per block (side-stream event, the operands the side stream reads), oldest first;
        # released in batches once the side stream has passed them (_release_side)
        pending: list = []
        # d: f32 gradient stream (residual accumulation); db: its bf16 copy, the GEMM operand (bf16 mode)
        d, db = K.pool_ln_bwd(dfeat.float(), *tape.pool, hn.weight, tape.out_shape, dlnw=g(hn.weight),
                              dlnb=g(hn.bias), with_bf16=bf)
        if tape.w2g_ready is not None:
            main.wait_event(tape.w2g_ready)
        self._ready([hn.weight, hn.bias])
        for st, (ds_saved, blocks_saved) in zip(reversed(list(self.stages)), reversed(tape.stages)):
            for bi in range(len(blocks_saved) - 1, -1, -1):
                blk, saved = st.blocks[bi], blocks_saved[bi]
                # the tape lets go of the block: its main-stream reads are stream-ordered before any
                # later main-stream allocation, its side-stream reads stay referenced below
                blocks_saved[bi] = None
                x, z, y, mean, rstd, gh, a = saved
                B, H, W, C = x.shape
                M = B * H * W
                d2 = d.view(M, C)
                w1 = self._w(blk.mlp.fc1.weight, cache)
                dsrc = db.view(M, C) if bf else d2
                if lean:
                    last = st is self.stages[0] and bi == 0
                    d, db = self._block_backward_lean(blk, saved, d, db, dsrc, cache, tape, main, side, pending, pol,
                                                      tail=tail if last and _TAIL_MAIN else None)
                    self._release_side(main, pending)
                    if last and _TAIL_MAIN == 2:
                        for job in tail:
                            job()
                        tail.clear()
                    continue
                # weight gradients (wgrad GEMMs, split-K reductions, depthwise wgrad) run on the side
                # stream beside the data-gradient chain of the main stream: the wgrads are MFMA-bound
                # with small outputs, the dgrads epilogue/HBM-bound, so the two overlap on the chip
                if side is not None:
                    side.wait_event(main.record_event())
                    for t_ in (dsrc, a):
                        t_.record_stream(side)
                with torch.cuda.stream(side) if side is not None else _nullctx():
                    # dW2 = gamma (.) d^T a, dgamma = rowdot(W2, d^T a) + b2 (.) colsum(d), db2 = gamma (.) colsum(d)
                    K.layerscale_wgrad(dsrc, a, blk.mlp.fc2.weight.detach(), blk.gamma.detach(),
                                       blk.mlp.fc2.bias.detach(), dw2=g(blk.mlp.fc2.weight), dgamma=g(blk.gamma),
                                       db2=g(blk.mlp.fc2.bias), compute_bf16=bf, policy=pol)
                ev_w2 = side.record_event() if side is not None else None
                # fc2: dh = ((d * gamma) @ W2) * GELU'(h).  bf16 mode folds gamma into a bf16 copy of W2;
                # GELU'(h) was stored by the forward epilogue
                dh = torch.empty(M, 4 * C, device=d.device, dtype=act)
                if bf:
                    w2g = tape.w2g.pop(id(blk), None)
                    if w2g is None:
                        w2g = K.scale_rows_bf16(blk.mlp.fc2.weight.detach(), blk.gamma.detach())
                    K.linear_dgrad(dsrc, w2g, out=dh, epilogue=nv.SV_EPI_MUL_AUX, aux=gh, compute_bf16=True, policy=pol)
                else:
                    K.linear_dgrad(d2, blk.mlp.fc2.weight.detach(), out=dh, epilogue=nv.SV_EPI_MUL_AUX,
                                   a_scale_k=blk.gamma, aux=gh, compute_bf16=False, policy=pol)
                # fc1: dy = dh @ W1 (main) ; dW1 = dh^T y, db1 = colsum(dh) (side, fused in the wgrad GEMM).
                # bf16 mode: dy and dz travel as bf16 (the depthwise backward reads dz through its LDS-DMA
                # ring, where 2-byte columns cost no more than 4-byte ones)
                if side is not None:
                    side.wait_event(main.record_event())
                    for t_ in (dh, y):
                        t_.record_stream(side)
                folds: list | None = [] if self.merge_folds else None  # one fold launch for the block
                with torch.cuda.stream(side) if side is not None else _nullctx():
                    K.linear_wgrad(dh, y, out=g(blk.mlp.fc1.weight), accumulate=True,
                                   bias_out=g(blk.mlp.fc1.bias), compute_bf16=bf, defer=folds, policy=pol)
                # bf16: the LayerNorm backward in the fc1 data gradient's epilogue where it applies (as the lean
                # schedule does, so both schedules give the same bits)
                fused = K.linear_dgrad_ln(dh, w1, z.view(M, C), mean, rstd, blk.norm.weight, dw=g(blk.norm.weight),
                                          db=g(blk.norm.bias), policy=pol) if bf else None
                if fused is not None:
                    dz, ln_finish = fused
                else:
                    dy = torch.empty(M, C, device=d.device, dtype=act)
                    K.linear_dgrad(dh, w1, out=dy, compute_bf16=bf, policy=pol)
                    # LayerNorm + depthwise conv; d += dwconv^T(dz) in place, bf16 copy refreshed (old copy dead)
                    # the LN weight/bias partials are folded on the side stream (off the data-gradient chain)
                    dz, ln_finish = K.layernorm_bwd(dy, z.view(M, C), mean, rstd, blk.norm.weight,
                                                    dw=g(blk.norm.weight), db=g(blk.norm.bias), out_dtype=act,
                                                    defer_reduce=True)
                dz4 = dz.view(B, H, W, C)
                blk_params = [blk.conv_dw.weight, blk.conv_dw.bias, blk.norm.weight, blk.norm.bias,
                              blk.mlp.fc1.weight, blk.mlp.fc1.bias, blk.mlp.fc2.weight, blk.mlp.fc2.bias, blk.gamma]
                if side is not None:
                    side.wait_event(main.record_event())
                    for t_ in (dz, x):
                        t_.record_stream(side)
                with torch.cuda.stream(side) if side is not None else _nullctx():
                    ln_finish(defer=folds)
                    K.dwconv7_bwd_weight(dz4, x, dw=g(blk.conv_dw.weight), db=g(blk.conv_dw.bias), defer=folds)
                    if folds is not None:
                        K.reduce_multi(folds)
                    # every gradient of the block is final on this stream now: the bucketer's event
                    # covers them all
                    self._ready(blk_params)
                if side is not None and bf:
                    # the bf16 copy of the gradient stream goes to a fresh buffer: the side stream's fc2
                    # wgrad may still be reading the previous one (record_stream above keeps it alive), so
                    # the main stream does not wait for the side stream here
                    db = torch.empty_like(db)
                elif side is not None:
                    main.wait_event(ev_w2)  # fp32: the fc2 wgrad reads d itself, which is updated in place
                K.dwconv7_bwd_data(dz4, blk.conv_dw.weight, d, accumulate=True, dx_bf16=db)
            if ds_saved is not None:
                x_prev, patches, d_mean, d_rstd = ds_saved
                ln, conv = st.downsample[0], st.downsample[1]
                B, H, W, C = x_prev.shape
                Cout = conv.weight.shape[0]
                Mo = B * (H // 2) * (W // 2)
                dsrc = db.view(Mo, Cout) if bf else d.view(Mo, Cout)
                wds = self._w(conv.weight, cache).reshape(Cout, 4 * C)
                dpatch = torch.empty(Mo, 4 * C, device=d.device, dtype=torch.float32)
                K.linear_dgrad(dsrc, wds, out=dpatch, compute_bf16=bf, policy=pol)
                K.linear_wgrad(dsrc, patches, out=g(conv.weight), accumulate=True, bias_out=g(conv.bias),
                               compute_bf16=bf, policy=pol)
                d, db = K.downsample_bwd(dpatch, x_prev, d_mean, d_rstd, ln.weight, dlnw=g(ln.weight),
                                         dlnb=g(ln.bias), with_bf16=bf)
                self._ready([ln.weight, ln.bias, conv.weight, conv.bias])
        conv, ln = self.stem[0], self.stem[1]
        if bf:
            # LayerNorm2d backward (f32 gradient stream, bf16 saved conv output) -> bf16 dz, then the
            # weight/bias gradient as one split-K wgrad GEMM over the saved patch rows (first 48 columns)
            patches, z0, s_mean, s_rstd = tape.stem
            C0 = conv.weight.shape[0]
            dz0 = K.layernorm_bwd(d.view(-1, C0), z0, s_mean, s_rstd, ln.weight, dw=g(ln.weight), db=g(ln.bias),
                                  out_dtype=torch.bfloat16)
            K.linear_wgrad(dz0, patches, out=g(conv.weight).view(C0, 48), accumulate=True, bias_out=g(conv.bias),
                           compute_bf16=True, cols=48, policy=pol)
        else:
            s_mean, s_rstd = tape.stem
            K.stem_bwd(tape.img, conv.weight, conv.bias, ln.weight, s_mean, s_rstd, d, dw=g(conv.weight),
                       db=g(conv.bias), dlnw=g(ln.weight), dlnb=g(ln.bias))
        for job in tail:
            job()
        if side is not None:
            main.wait_stream(side)  # clip / AdamW / the next step see every side-stream gradient
            pending.clear()  # safe: later main-stream allocations are ordered after the join
        self._ready([conv.weight, conv.bias, ln.weight, ln.bias])


    # lean mode keeps at most 2 x _RELEASE_BATCH blocks of side-stream operands (dh alone is M x 4C
    # bf16) instead of every block's until the backward ends; one main->side wait per batch
    _RELEASE_BATCH = int(os.environ.get("SV_RELEASE_BATCH", "4"))

    @classmethod
    def _release_side(cls, main, pending: list) -> None:
        """Drop the side-stream operands of the oldest blocks: free ones whose event has completed,
        and once 2 x _RELEASE_BATCH blocks are pending, make main wait for the side stream to pass
        the oldest batch (cheap: the side stream runs about one block behind) and drop that batch."""
        while pending and pending[0][0].query():
            pending.pop(0)
        if len(pending) >= 2 * cls._RELEASE_BATCH:
            main.wait_event(pending[cls._RELEASE_BATCH - 1][0])
            del pending[:cls._RELEASE_BATCH]

    def _block_backward_lean(self, blk, saved, d, db, dsrc, cache, tape, main, side, pending, pol, tail=None):
        """bf16 block backward with one main->side hand-off.  Main: fc2 dgrad (x GELU'), fc1 dgrad,
        LayerNorm backward, depthwise backward-data.  Side, after the LayerNorm backward: fc2 wgrad
        (+ gamma, bias), fc1 wgrad (+ bias), the LayerNorm weight/bias fold and the depthwise wgrad of
        the block, beside the main stream's next block.  ``pol``: the main stream's GEMM policy; the side
        stream's GEMMs run at raised wave priority where they share a CU with the main stream's data-gradient
        GEMMs (+1.0% step, interleaved A/B gpurun_out prio2; raising the main stream's instead cost 0.7%,
        prio1), under side_grid_cap when set.  Returns the new (d, db).

        ``tail`` (the backward's last block): the side stream, about one block behind the main stream, would run
        this block's three weight gradients after the main stream has finished (the step's end waited ~0.5 ms on
        it, r11k trace); only the fc2 one goes there, and the fc1 and depthwise ones (with the block's fold) are
        appended to ``tail`` for the main stream to run after the stem."""
        g = self._grad
        x, z, y, mean, rstd, gh, a = saved
        B, H, W, C = x.shape
        M = B * H * W
        wt = tape.wt.pop(id(blk), None)
        dh = torch.empty(M, 4 * C, device=d.device, dtype=torch.bfloat16)
        if wt is not None:
            # fused: fc2 data gradient (x GELU') -> fc1 data gradient -> LayerNorm backward in one kernel
            dz = torch.empty(M, C, device=d.device, dtype=torch.bfloat16)
            part, P = K.mlp_bwd(dsrc, wt[0], gh, wt[1], z.view(M, C), mean, rstd, blk.norm.weight, dh=dh, dz=dz)
            dw_ln, db_ln = g(blk.norm.weight), g(blk.norm.bias)

            def ln_finish(record: bool = True, defer: list | None = None, _p=part, _n=P):
                if defer is not None:
                    defer += [(_p[0], dw_ln, _n, True), (_p[1], db_ln, _n, True)]
                else:
                    K.reduce_pair(_p[0], dw_ln, _p[1], db_ln, _n)
        else:
            w1 = self._w(blk.mlp.fc1.weight, cache)
            w2g = tape.w2g.pop(id(blk), None)
            if w2g is None:
                w2g = K.scale_rows_bf16(blk.mlp.fc2.weight.detach(), blk.gamma.detach())
            K.linear_dgrad(dsrc, w2g, out=dh, epilogue=nv.SV_EPI_MUL_AUX, aux=gh, compute_bf16=True, policy=pol)
            # fc1 data gradient with the LayerNorm backward in its epilogue (C = 512 / 1024: dy never reaches HBM);
            # None where the fused form does not apply -> the two passes
            fused = K.linear_dgrad_ln(dh, w1, z.view(M, C), mean, rstd, blk.norm.weight, dw=g(blk.norm.weight),
                                      db=g(blk.norm.bias), policy=pol)
            if fused is not None:
                dz, ln_finish = fused
            else:
                dy = torch.empty(M, C, device=d.device, dtype=torch.bfloat16)
                K.linear_dgrad(dh, w1, out=dy, compute_bf16=True, policy=pol)
                dz, ln_finish = K.layernorm_bwd(dy, z.view(M, C), mean, rstd, blk.norm.weight, dw=g(blk.norm.weight),
                                                db=g(blk.norm.bias), out_dtype=torch.bfloat16, defer_reduce=True)
        dz4 = dz.view(B, H, W, C)
        nv.handoff(main, side)
        # the main stream's next launch is enqueued first: the depthwise backward-data needs only dz, and the host's
        # side-stream enqueues below left the main queue idle ~18 us per block before it (r13n trace, queue_gaps.py).
        # The side stream still reads dsrc (this block's bf16 gradient copy): the next copy gets a fresh buffer
        db = torch.empty_like(db)
        K.dwconv7_bwd_data(dz4, blk.conv_dw.weight, d, accumulate=True, dx_bf16=db)
        side_cap = pol.grid_cap
        if self.side_grid_cap is not None:
            side_cap = min(self.side_grid_cap, side_cap) if side_cap > 0 else self.side_grid_cap
        spol = nv.policy(impl=self.side_impl, grid_cap=side_cap, wg_per_cu=pol.wg_per_cu, priority=self.side_prio)
        def rest(policy):
            # the block's remaining folds (fc1 wgrad slab + bias, LayerNorm and depthwise weight / bias
            # partials) in ONE launch instead of four
            folds: list | None = [] if self.merge_folds else None
            K.linear_wgrad(dh, y, out=g(blk.mlp.fc1.weight), accumulate=True, bias_out=g(blk.mlp.fc1.bias),
                           compute_bf16=True, defer=folds, policy=policy, wgrad_target=self.wgrad_target)
            ln_finish(record=False, defer=folds)
            K.dwconv7_bwd_weight(dz4, x, dw=g(blk.conv_dw.weight), db=g(blk.conv_dw.bias), defer=folds)
            if folds is not None:
                K.reduce_multi(folds)
            return folds

        with torch.cuda.stream(side):
            K.layerscale_wgrad(dsrc, a, blk.mlp.fc2.weight.detach(), blk.gamma.detach(), blk.mlp.fc2.bias.detach(),
                               dw2=g(blk.mlp.fc2.weight), dgamma=g(blk.gamma), db2=g(blk.mlp.fc2.bias),
                               compute_bf16=True, policy=spol, wgrad_target=self.wgrad_target)
            if tail is None:
                folds = rest(spol)
                self._ready([blk.conv_dw.weight, blk.conv_dw.bias, blk.norm.weight, blk.norm.bias,
                             blk.mlp.fc1.weight, blk.mlp.fc1.bias, blk.mlp.fc2.weight, blk.mlp.fc2.bias, blk.gamma])
            else:
                folds = None
                self._ready([blk.mlp.fc2.weight, blk.mlp.fc2.bias, blk.gamma])
            pending.append((side.record_event(), (dsrc, dh, dz, ln_finish, x, y, a, folds)))
        if tail is not None:
            def job(_rest=rest, _pol=pol):
                _rest(_pol)
                self._ready([blk.conv_dw.weight, blk.conv_dw.bias, blk.norm.weight, blk.norm.bias,
                             blk.mlp.fc1.weight, blk.mlp.fc1.bias])
            tail.append(job)
        return d, db


def create_convnext(name: str, precision: str = "bf16") -> ConvNeXtHip:
    key = name.split(".")[0]
    if key not in CONVNEXT_CFGS:
        raise ValueError(f"unsupported ConvNeXt variant {name!r}")
    depths, dims = CONVNEXT_CFGS[key]
    return ConvNeXtHip(depths, dims, precision=precision)
