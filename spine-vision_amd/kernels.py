"""Typed host-side launch helpers over the C ABI (``include/sv_kernels.h``).

Every helper takes/returns torch device tensors, validates shapes on the host *before* launching
(the kernels assume the grid/shape contract checked here), allocates outputs and workspaces from
PyTorch's caching allocator and enqueues on the current stream.  There is no fallback path: a
missing library or a CPU tensor raises.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import native as nv
from .native import SV_BF16, SV_F32, call, dt, ptr, value

EPS_LN = 1e-6


class GemmProbe:
    """Times every launch of one GEMM class with HIP events on the launching stream (bench.py's live
    roofline measurement).  key = (a_kmajor, b_kmajor, compute_bf16) or, to single out one epilogue
    kind, (a_kmajor, b_kmajor, compute_bf16, epilogue).  ``bytes`` counts the ALGORITHMIC HBM bytes
    of the launch: operands read once (A, B, the epilogue operand) and the REQUIRED outputs written
    once -- for a split-K weight gradient that is the N x K f32 gradient, not the self-chosen slabs."""

    def __init__(self, key: tuple, name: str = "") -> None:
        self.key = key
        self.name = name
        self.events: list[tuple[torch.cuda.Event, torch.cuda.Event]] = []
        self.flops = 0.0
        self.bytes = 0.0
        self.launches = 0
        # per launch: the fraction of the chip's CUs its grid is sized for (256x256 tiles x split-K slices, capped
        # by the policy's grid cap), so a class that runs on part of the chip by design can be read against the
        # peak of the CUs it was given (bench.py: frac_of_granted_cus)
        self.shares: list[float] = []

    def matches(self, a_kmajor: bool, b_kmajor: bool, bf: bool, epilogue: int) -> bool:
        k = (bool(a_kmajor), bool(b_kmajor), bool(bf))
        return self.key[:3] == k and (len(self.key) < 4 or self.key[3] == epilogue)

    def elapsed_ms(self) -> float:
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.events)


PROBES: list[GemmProbe] = []
# single-probe alias kept for older tools (tools/*.py set K.PROBE)
PROBE: GemmProbe | None = None


class OpProbe:
    """Times every launch of one HBM-bound kernel (depthwise conv fwd / bwd-data / wgrad, LayerNorm
    backward, AdamW) with HIP events on the launching stream; ``bytes`` are the kernel's ALGORITHMIC HBM
    bytes (every operand read once, every required output written once; partial sums it chooses to
    write for a later fold are not counted)."""

    def __init__(self, name: str) -> None:
        self.name = name
        self.events: list = []
        self.flops = 0.0
        self.bytes = 0.0
        self.fma = 0.0  # f32 VALU FMAs (the depthwise convolutions: 49 per output element)
        self.launches = 0

    def elapsed_ms(self) -> float:
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.events)


OP_PROBES: dict[str, OpProbe] = {}  # name -> probe; bench.py fills it for the timed step it probes


# SV_DIAG_SKIP=fold,...: skip every launch of those probe classes (an upper bound on what removing them could buy;
# the step's results are wrong -- never for training or tests)
_DIAG_SKIP = {x for x in os.environ.get("SV_DIAG_SKIP", "").split(",") if x}


def _fin(name: str, *args) -> None:
    """call() of a BatchNorm fold / activation launch; SV_DIAG_SKIP=bn_fin / bn_act skips those (diagnostic only)"""
    if _DIAG_SKIP and not name.endswith("_fold") and ("bn_act" if name == "sv_bn_act_fwd" else "bn_fin") in _DIAG_SKIP:
        return
    call(name, *args)


def _timed_call(op: str, nbytes: float, *args, fma: float = 0.0, flops: float = 0.0) -> None:
    """call(*args), bracketed by HIP events on the current stream when ``op`` is being probed; ``fma``: the
    launch's algorithmic f32 VALU FMAs (its roof when they outlast its bytes)."""
    if _DIAG_SKIP and op in _DIAG_SKIP:  # diagnostic timing only: the launch is skipped, its results are garbage
        return
    pr = OP_PROBES.get(op)
    if pr is None:
        call(*args)
        return
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    call(*args)
    ev1.record()
    pr.events.append((ev0, ev1))
    pr.bytes += nbytes
    pr.fma += fma
    pr.flops += flops
    pr.launches += 1


_CUS: dict = {}


def _device_cus(device) -> int:
    n = _CUS.get(device)
    if n is None:
        n = _CUS[device] = torch.cuda.get_device_properties(device).multi_processor_count
    return n


def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def _cdt(compute_bf16: bool) -> int:
    return SV_BF16 if compute_bf16 else SV_F32


# ----------------------------------------------------------------------------------------------
# GEMM
def gemm(
    A: torch.Tensor,
    B: torch.Tensor,
    *,
    M: int,
    N: int,
    K: int,
    a_kmajor: bool,
    b_kmajor: bool,
    lda: int,
    ldb: int,
    epilogue: int = nv.SV_EPI_STORE,
    C: torch.Tensor | None = None,
    C2: torch.Tensor | None = None,
    ldc: int | None = None,
    bias: torch.Tensor | None = None,
    gamma: torch.Tensor | None = None,
    aux: torch.Tensor | None = None,
    ld_aux: int | None = None,
    a_scale_k: torch.Tensor | None = None,
    split_k: int = 1,
    compute_bf16: bool = True,
    bn: "nv.BnRef | None" = None,
    policy: "nv.GemmPolicy | None" = None,
    fold: tuple | None = None,
) -> torch.Tensor:
    """C = epilogue(A(m,k) . B(k,n)); see sv_gemm in include/sv_kernels.h for the layouts.  ``policy``: the
    launch policy of this call (nv.policy(...): kernel family, grid cap, residency, priority); None = defaults."""
    _check(C is not None, "gemm: output tensor C is required")
    need_a = (M - 1) * lda + K if a_kmajor else (K - 1) * lda + M
    need_b = (N - 1) * ldb + K if b_kmajor else (K - 1) * ldb + N
    _check(A.numel() >= need_a, f"gemm: A too small ({A.numel()} < {need_a})")
    _check(B.numel() >= need_b, f"gemm: B too small ({B.numel()} < {need_b})")
    if epilogue == nv.SV_EPI_SLAB:
        _check(C.dtype in (torch.float32, torch.bfloat16) and C.numel() >= split_k * M * N, "gemm: slab too small")
    else:
        ldc = N if ldc is None else ldc
        _check(C.numel() >= (M - 1) * ldc + N, "gemm: C too small")
    if bias is not None:
        _check(bias.numel() >= N and bias.dtype == torch.float32, "gemm: bad bias")
    d = nv.GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.a_dtype, d.a_kmajor, d.lda = ptr(A), dt(A), int(a_kmajor), lda
    d.B, d.b_dtype, d.b_kmajor, d.ldb = ptr(B), dt(B), int(b_kmajor), ldb
    d.a_scale_k = ptr(a_scale_k)
    d.epilogue = epilogue
    d.C, d.c_dtype, d.ldc = ptr(C), dt(C), ldc if ldc is not None else N
    if C2 is not None:
        d.C2, d.c2_dtype = ptr(C2), dt(C2)
    d.bias = ptr(bias)
    d.gamma = ptr(gamma)
    if aux is not None:
        d.aux, d.aux_dtype, d.ld_aux = ptr(aux), dt(aux), ld_aux if ld_aux is not None else N
    d.split_k = split_k
    d.compute = _cdt(compute_bf16)
    if bn is not None:
        d.bn = ctypes.pointer(bn)
    if policy is not None:
        d.policy = policy
    if fold is not None:  # (out, accumulate, counters): the split-K fold inside the GEMM (SV_EPI_SLAB)
        fo, facc, fcnt = fold
        d.fold_out, d.fold_ld, d.fold_accumulate, d.fold_counters = ptr(fo), N, int(bool(facc)), ptr(fcnt)
    probes = [p_ for p_ in (PROBES + ([PROBE] if PROBE is not None else [])) if p_.matches(a_kmajor, b_kmajor,
                                                                                      compute_bf16, epilogue)]
    if probes:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        call("sv_gemm", ctypes.byref(d))
        ev1.record()
        nbytes = M * K * A.element_size() + N * K * B.element_size()
        if epilogue == nv.SV_EPI_SLAB:
            nbytes += M * N * 4  # the weight gradient itself (the split-K slabs are a design choice)
            if C2 is not None:
                nbytes += M * 4  # its bias gradient (column sums)
        elif epilogue == nv.SV_EPI_BIAS_GELU_DUAL:
            nbytes += M * N * C2.element_size()  # GELU(h) is required; the GELU'(h) store is a design choice
        elif epilogue == nv.SV_EPI_LN_BWD:
            nbytes += M * N * C.element_size() + M * 8 + C2.numel() * 4  # dz; mean / rstd; the weight / bias partials
        else:
            nbytes += M * N * C.element_size()
            if C2 is not None:
                nbytes += M * N * C2.element_size()
        if aux is not None:
            nbytes += M * N * aux.element_size()
        cus = _device_cus(C.device)
        cap = policy.grid_cap if policy is not None and policy.grid_cap > 0 else cus
        share = min(-(-M // 256) * -(-N // 256) * max(split_k, 1), cap, cus) / cus
        for p_ in probes:
            p_.events.append((ev0, ev1))
            p_.shares.append(share)
            p_.flops += 2.0 * M * N * K
            p_.bytes += nbytes
            p_.launches += 1
    else:
        call("sv_gemm", ctypes.byref(d))
    return C


# the LayerNorm backward in the fc1 data gradient's epilogue (SV_EPI_LN_BWD, round 6): dy never reaches HBM.  v9 only,
# N % 256 == 0 (ConvNeXt C = 512 / 1024), every 256x256 tile resident at once (else the two-pass form runs).
# SV_FUSED_LN_BWD=0 keeps the two passes (A/B runs)
FUSED_LN_BWD = os.environ.get("SV_FUSED_LN_BWD", "1") != "0"
_LN_XCH: dict = {}


def linear_dgrad_ln(dh2d, w, z2d, mean, rstd, lnw, *, dw, db, policy=None):
    """dz = LayerNorm backward of dy = bf16(dh2d @ w) over (z2d, mean, rstd, lnw) in ONE launch (sv_gemm,
    SV_EPI_LN_BWD); -> (dz bf16 [M, C], finish) as layernorm_bwd(..., defer_reduce=True) returns, or None where the
    shape or the chip's free CUs do not take the fused form (the caller then runs linear_dgrad + layernorm_bwd)."""
    if not FUSED_LN_BWD:
        return None
    M, K = dh2d.shape
    C = w.shape[1]
    if C % 256 or C > 1024 or dh2d.dtype != torch.bfloat16 or z2d.dtype != torch.bfloat16:
        return None
    _check(tuple(z2d.shape) == (M, C) and z2d.is_contiguous() and mean.numel() == M and rstd.numel() == M
           and lnw.numel() == C, "linear_dgrad_ln: z [M, C], mean / rstd [M], lnw [C]")
    tilesM, tilesN = -(-M // 256), C // 256
    if tilesM * tilesN > _device_cus(dh2d.device):
        return None
    dz = torch.empty(M, C, device=dh2d.device, dtype=torch.bfloat16)
    P = -(-M // 128)
    part = torch.empty(2, P, C, device=dh2d.device, dtype=torch.float32)
    key = (dh2d.device, nv._stream())
    xch = _LN_XCH.get(key)
    if xch is None or xch.numel() < tilesM * tilesN * 512:
        xch = _LN_XCH[key] = torch.empty(max(tilesM * tilesN * 512, 1 << 18), device=dh2d.device, dtype=torch.float32)
    bn = nv.BnRef(ptr(mean), ptr(rstd), ptr(lnw), None)
    try:
        gemm(dh2d, w, M=M, N=C, K=K, a_kmajor=True, b_kmajor=False, lda=K, ldb=C, epilogue=nv.SV_EPI_LN_BWD, C=dz,
             C2=part, aux=z2d, ld_aux=C, compute_bf16=True, bn=bn, policy=policy,
             fold=(xch, False, _fold_counters(dh2d.device, tilesM)))
    except RuntimeError as err:
        if "(status 2)" in str(err):  # SV_ERR_UNSUPPORTED: not every tile resident at once (CU mask, grid cap)
            return None
        raise

    def finish(record: bool = True, defer: list | None = None):
        if record:
            part.record_stream(torch.cuda.current_stream())
        if defer is not None:
            defer += [(part[0], dw, P, True), (part[1], db, P, True)]
            return
        reduce_pair(part[0], dw, part[1], db, P)

    return dz, finish


def linear_fwd(x2d, w, *, out, bias=None, epilogue=nv.SV_EPI_STORE, out2=None, gamma=None, residual=None,
               compute_bf16=True, policy=None):
    """out[M,N] = epilogue(x2d[M,K] @ w[N,K]^T)  (torch Linear weight layout)."""
    M, K = x2d.shape
    N = w.shape[0]
    return gemm(x2d, w, M=M, N=N, K=K, a_kmajor=True, b_kmajor=True, lda=K, ldb=K, epilogue=epilogue, C=out,
                C2=out2, bias=bias, gamma=gamma, aux=residual, compute_bf16=compute_bf16, policy=policy)


def linear_dgrad(dy2d, w, *, out, epilogue=nv.SV_EPI_STORE, a_scale_k=None, aux=None, compute_bf16=True, policy=None):
    """out[M,K] = epilogue((dy2d[M,N] * a_scale_k[N]) @ w[N,K])."""
    M, N = dy2d.shape
    K = w.shape[1]
    return gemm(dy2d, w, M=M, N=K, K=N, a_kmajor=True, b_kmajor=False, lda=N, ldb=K, epilogue=epilogue, C=out,
                a_scale_k=a_scale_k, aux=aux, compute_bf16=compute_bf16, policy=policy)


# channel counts the fused MLP forward kernel (csrc/mlp.hip) is built for: ConvNeXt-base S1 / S2, ConvNeXt-large S1
MLP_FUSED_C = (128, 192, 256, 512)


def mlp_fwd(y, w1, b1, w2, b2, gamma, x, *, out, gelu_grad=None, gelu_out=None):
    """Fused ConvNeXt MLP forward (sv_mlp_fwd): out = gamma (.) (GELU(y w1^T + b1) w2^T + b2) + x in one kernel,
    the 4C-wide hidden activation kept on chip; ``gelu_grad`` / ``gelu_out`` ([M, 4C] bf16, both or neither) receive
    GELU'(h) / GELU(h) for the backward (training).  Bit for bit the two-GEMM path (linear_fwd GELU dual, then the
    gamma-residual epilogue)."""
    M, C = y.shape
    H = 4 * C
    _check(C in MLP_FUSED_C, f"mlp_fwd: C = {C} not supported {MLP_FUSED_C}")
    _check(y.dtype == torch.bfloat16 and w1.dtype == torch.bfloat16 and w2.dtype == torch.bfloat16,
           "mlp_fwd: y / w1 / w2 must be bf16")
    _check(tuple(w1.shape) == (H, C) and tuple(w2.shape) == (C, H), "mlp_fwd: weight shapes")
    for t_, n_ in ((b1, H), (b2, C), (gamma, C)):
        _check(t_.dtype == torch.float32 and t_.numel() == n_ and t_.is_contiguous(), "mlp_fwd: bias / gamma")
    _check(x.dtype == torch.float32 and out.dtype == torch.float32 and x.numel() == M * C and out.numel() == M * C,
           "mlp_fwd: x / out must be f32 [M, C]")
    _check(out.data_ptr() != x.data_ptr(), "mlp_fwd: out must not alias x")
    _check((gelu_grad is None) == (gelu_out is None), "mlp_fwd: gelu_grad and gelu_out go together")
    ts = [y, w1, b1, w2, b2, gamma, x, out]
    if gelu_grad is not None:
        for t_ in (gelu_grad, gelu_out):
            _check(t_.dtype == torch.bfloat16 and t_.numel() == M * H, "mlp_fwd: GELU outputs must be bf16 [M, 4C]")
        ts += [gelu_grad, gelu_out]
    _check(all(t_.is_contiguous() and t_.data_ptr() % 16 == 0 for t_ in ts), "mlp_fwd: contiguous 16-B aligned tensors")
    _check(M * H * 2 < 2**31, "mlp_fwd: hidden tensor must be < 2 GiB")
    # algorithmic: y, x read; out written; both weights once; the GELU pair written in training
    nb = M * C * (2 + 4 + 4) + 2 * H * C * 2 + (2 * M * H * 2 if gelu_grad is not None else 0)
    _timed_call("mlp_fused", nb, "sv_mlp_fwd", ptr(y), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(gamma), ptr(x), ptr(out),
                ptr(gelu_grad), ptr(gelu_out), M, C, flops=4.0 * M * C * H)
    return out


def transpose_scale_bf16(W: torch.Tensor, scale: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """bf16(W * scale[:, None])^T for a 2-D f32 weight [R, C] -> [C, R] bf16 (the operand images of mlp_bwd)."""
    R_, C_ = W.shape
    _check(W.dtype == torch.float32 and W.is_contiguous(), "transpose_scale_bf16: need contiguous f32")
    _check(scale is None or (scale.numel() == R_ and scale.dtype == torch.float32), "transpose_scale_bf16: bad scale")
    if out is None:
        out = torch.empty(C_, R_, device=W.device, dtype=torch.bfloat16)
    _check(tuple(out.shape) == (C_, R_) and out.dtype == torch.bfloat16 and out.is_contiguous(),
           "transpose_scale_bf16: bad out")
    call("sv_transpose_scale_bf16", ptr(W), ptr(scale), ptr(out), R_, C_)
    return out


MLP_BWD_FUSED_C = (128,)


def mlp_bwd(d, w2t, gelu_grad, w1t, z, mean, rstd, lnw, *, dh, dz):
    """Fused backward of fc2 (x GELU') -> fc1 -> LayerNorm of a ConvNeXt block at C = 128 (sv_mlp_bwd): dh (bf16
    [M, 4C], bit for bit linear_dgrad(d, W2 gamma, x GELU')), dz (bf16 [M, C], the LayerNorm backward of bf16(dh W1)).
    Returns the LayerNorm weight / bias partial sums (ln_part [2][P][C] f32) and P, to fold into dw / db."""
    M, C = d.shape
    H = 4 * C
    _check(C in MLP_BWD_FUSED_C, f"mlp_bwd: C = {C} not supported {MLP_BWD_FUSED_C}")
    for t_, shp in ((d, (M, C)), (w2t, (H, C)), (gelu_grad, (M, H)), (w1t, (C, H)), (z, (M, C)), (dh, (M, H)),
                    (dz, (M, C))):
        _check(t_.dtype == torch.bfloat16 and t_.numel() == shp[0] * shp[1] and t_.is_contiguous(),
               f"mlp_bwd: bf16 [{shp[0]}, {shp[1]}] operand expected")
    for t_, n_ in ((mean, M), (rstd, M), (lnw, C)):
        _check(t_.dtype == torch.float32 and t_.numel() == n_ and t_.is_contiguous(), "mlp_bwd: f32 vector")
    P = value("sv_mlp_bwd_nparts", M, C)
    part = torch.empty(2, P, C, device=d.device, dtype=torch.float32)
    ts = [d, w2t, gelu_grad, w1t, z, mean, rstd, lnw, dh, dz, part]
    _check(all(t_.data_ptr() % 16 == 0 for t_ in ts), "mlp_bwd: 16-B aligned tensors")
    _check(M * H * 2 < 2**31, "mlp_bwd: hidden tensor must be < 2 GiB")
    # algorithmic: d, GELU'(h), z read; dh, dz written; both weights, mean / rstd once
    nb = M * (C * 2 + H * 2 + C * 2 + H * 2 + C * 2 + 8) + 2 * H * C * 2
    _timed_call("mlp_bwd_fused", nb, "sv_mlp_bwd", ptr(d), ptr(w2t), ptr(gelu_grad), ptr(w1t), ptr(z), ptr(mean),
                ptr(rstd), ptr(lnw), ptr(dh), ptr(dz), ptr(part), M, C, flops=4.0 * M * C * H)
    return part, P


_WGRAD_TARGET = 512  # workgroups per split-K wgrad launch (2 per CU)
# persistent 256x256 wgrads: tiles x split ~ this many workgroups (SV_WGRAD9_WGS for A/B runs).  Half the chip
# (128): the side-stream weight gradients share it with the main stream's data gradients anyway, and half the
# split depth halves the f32 slabs written and folded -- round 4 on the final kernels: 1072.6-1075.6 vs
# 1065.7-1067.9 img/s interleaved, fold 4.0 -> 2.5 ms/step (profiles/round4/r7f_fold_ab.txt; round 3 had
# measured 128 and 256 equal)
_WGRAD9_TARGET = int(os.environ.get("SV_WGRAD9_WGS", "128"))
# ...but the whole chip for long weight gradients: ConvNeXt-large bs64's (309 GFLOP each) on half the chip made the
# side stream the long pole (590 vs 598 img/s at 256, profiles/round4/r9c_large_wgrad_target.txt)
_WGRAD9_LONG_GFLOP = float(os.environ.get("SV_WGRAD9_LONG_GFLOP", "150"))


def _wgrad_split(tiles: int, K: int) -> int:
    """K slices so that tiles*split ~ 512 workgroups (2 per CU), each slice >= 16 k-steps."""
    split = max(1, -(-_WGRAD_TARGET // max(tiles, 1)))
    return max(1, min(split, K // 512 if K >= 512 else 1))


def _wgrad_split_for(N: int, K: int, M: int, target: int | None = None) -> int:
    """Split-K factor of a weight gradient G[N,K] = dY[M,N]^T X[M,K].  Outputs of at least 128 x 256 run
    on the persistent 256x256 kernel (gemm9.hip; a 128-row output half-fills its tiles and still beats
    the 256x128 kernel): one tile per CU (tiles * split ~ 256 CUs) with every K slice a whole number of
    64-deep K-tiles; smaller ones on the 256x128 kernel (~512 workgroups)."""
    if min(N, K) >= 128 and max(N, K) >= 256:
        tiles9 = -(-N // 256) * -(-K // 256)
        target = (target or _WGRAD9_TARGET) if 2.0 * M * N * K <= _WGRAD9_LONG_GFLOP * 1e9 else 256
        # the slice count whose grid is nearest the target, among those that cut M into whole 64-row K-tiles and
        # keep one workgroup per CU (rounding down alone left ConvNeXt-large's S3 wgrads, 36 tiles, at split 2:
        # 72 workgroups, 47 % longer launches, the large bs64 step 16 % slower, profiles/round4/r9b_configs/)
        ok = [s_ for s_ in range(1, max(2, 2 * target // tiles9 + 1)) if M % (s_ * 64) == 0 and tiles9 * s_ <= 256]
        if ok:
            return min(ok, key=lambda s_: (abs(tiles9 * s_ - target), s_))
    return _wgrad_split(-(-N // 128) * -(-K // 128), M)


# In-kernel split-K fold of the weight gradients (gemm9.hip, sv_gemm_desc.fold_out), where the separate fold would
# take sv_reduce_partials' sequential wide body (bitwise the same result).  The kernel spreads each tile's fold over
# the tile's own slices when the grid allows it (every slice resident: one unit per workgroup, at most half the
# CUs), else the last workgroup to finish a slice sums the tile.  Opt-in (SV_INKERNEL_FOLD=1), both forms measured
# slower in the step: the last-arriver form 1009-1051 vs 1066-1068 img/s (r7f_fold_ab.txt: one CU streams the
# tile), the spread form 1037-1039 vs 1056-1057 (r8j_spread_fold_ab.txt: the fold passes drop 2.4 -> 1.7 ms/step
# but each wgrad launch grows 170 -> 195 us in-step, its slices waiting on one another beside the main stream)
_INKERNEL_FOLD = os.environ.get("SV_INKERNEL_FOLD", "0") != "0"
_FOLD_MAX_SPLIT = int(os.environ.get("SV_FOLD_MAX_SPLIT", "64"))
_FOLD_COUNTERS: dict = {}


def _fold_counters(device, tiles: int) -> torch.Tensor:
    """Zeroed int32 counters (arrivals, departures) per tile for in-kernel folds on the current stream (the kernel
    leaves them zero)."""
    key = (device, nv._stream())
    t = _FOLD_COUNTERS.get(key)
    if t is None or t.numel() < 2 * tiles:
        t = _FOLD_COUNTERS[key] = torch.zeros(max(2 * tiles, 4096), device=device, dtype=torch.int32)
    return t


# bf16 split-K slabs for the v9 weight gradients: each slice's f32 partial rounded to bf16 once (the reference's
# autocast rounds the whole weight gradient to bf16 once), summed in f32 in slice order by the fold -- half the slab
# bytes written and read.  ConvNeXt-base bs32 +1.5 % (1091-1098 vs 1077-1079 img/s interleaved), its B=32 parity
# against the fp32 oracle unchanged (worst gradient 7.89e-3 vs 7.9e-3; profiles/round4/r9zh_bf16_slabs_ab.txt).
# SV_WGRAD_BF16_SLABS=0: f32 slabs.  Only the default / v9 kernel family (policy.impl 0 or 9) takes them.
_WGRAD_BF16_SLABS = os.environ.get("SV_WGRAD_BF16_SLABS", "1") != "0"


def _bf16_slabs(N: int, K: int, M: int, split: int, compute_bf16: bool, policy=None) -> bool:
    """the v9 weight-gradient shapes (whole 64-row K-tiles per slice: _wgrad_split_for's v9 branch)"""
    return (_WGRAD_BF16_SLABS and compute_bf16 and split > 1 and min(N, K) >= 128 and max(N, K) >= 256
            and K % 8 == 0 and M % (split * 64) == 0 and (policy is None or policy.impl in (0, 9)))


def _fold_ok(split: int, n: int, out: torch.Tensor, compute_bf16: bool) -> bool:
    return (_INKERNEL_FOLD and compute_bf16 and 1 < split <= _FOLD_MAX_SPLIT and n >= 65536 and n % 4 == 0
            and out.dtype == torch.float32 and out.is_contiguous() and out.data_ptr() % 16 == 0)


def linear_wgrad(dy2d, x2d, *, out=None, accumulate=False, bias_out=None, bias_accumulate=True,
                 compute_bf16=True, cols=None, defer: list | None = None, policy=None,
                 wgrad_target: int | None = None) -> torch.Tensor:
    """G[N,K] = dy2d[M,N]^T @ x2d[M,K] in f32 (split-K over M into slabs, then one reduce pass that
    writes -- or, with ``accumulate``, adds -- into ``out``).  With ``bias_out`` the column sums of
    dy2d (the bias gradient) come out of the same GEMM (SV_EPI_SLAB colsum).  ``cols``: use only the
    first ``cols`` columns of x2d (the stem's 48 of its 64-wide padded patch rows).  ``defer`` (a list, with
    ``out`` given): append the slab folds to it for one ``reduce_multi`` launch instead of reducing here."""
    M, N = dy2d.shape
    ldx = x2d.shape[1]
    K = ldx if cols is None else cols
    split = _wgrad_split_for(N, K, M, wgrad_target)
    cs = torch.empty(split * N, device=dy2d.device, dtype=torch.float32) if bias_out is not None else None
    if (out is not None and _bf16_slabs(N, K, M, split, compute_bf16, policy) and out.is_contiguous()
            and out.numel() == N * K):
        slab16 = torch.empty(split * N * K, device=dy2d.device, dtype=torch.bfloat16)
        gemm(dy2d, x2d, M=N, N=K, K=M, a_kmajor=False, b_kmajor=False, lda=N, ldb=ldx, epilogue=nv.SV_EPI_SLAB,
             C=slab16, C2=cs, split_k=split, compute_bf16=True, policy=policy)
        _timed_call("fold", 2.0 * split * N * K + 4.0 * N * K * (1 + int(bool(accumulate))), "sv_reduce_partials_bf16",
                    ptr(slab16), split, N * K, ptr(out), 1.0, int(bool(accumulate)))
        if cs is not None:
            if defer is not None:
                defer.append((cs, bias_out, split, bias_accumulate))
            else:
                reduce_into(cs, split, bias_out, accumulate=bias_accumulate)
        return out
    slab = torch.empty(split * N * K, device=dy2d.device, dtype=torch.float32)
    if out is not None and _fold_ok(split, N * K, out, compute_bf16):
        _check(out.numel() == N * K, "linear_wgrad: bad out")
        gemm(dy2d, x2d, M=N, N=K, K=M, a_kmajor=False, b_kmajor=False, lda=N, ldb=ldx, epilogue=nv.SV_EPI_SLAB,
             C=slab, C2=cs, split_k=split, compute_bf16=compute_bf16, policy=policy,
             fold=(out, accumulate, _fold_counters(dy2d.device, -(-N // 256) * -(-K // 256))))
        if cs is not None:
            if defer is not None:
                defer.append((cs, bias_out, split, bias_accumulate))
            else:
                reduce_into(cs, split, bias_out, accumulate=bias_accumulate)
        return out
    gemm(dy2d, x2d, M=N, N=K, K=M, a_kmajor=False, b_kmajor=False, lda=N, ldb=ldx, epilogue=nv.SV_EPI_SLAB,
         C=slab, C2=cs, split_k=split, compute_bf16=compute_bf16, policy=policy)
    if out is None:
        if split == 1 and not accumulate:
            if cs is not None:
                reduce_into(cs, split, bias_out, accumulate=bias_accumulate)
            return slab.view(N, K)
        out = torch.empty(N, K, device=dy2d.device, dtype=torch.float32)
        accumulate = False
    _check(out.numel() == N * K and out.is_contiguous(), "linear_wgrad: bad out")
    if defer is not None:
        defer.append((slab, out, split, accumulate))
        if cs is not None:
            defer.append((cs, bias_out, split, bias_accumulate))
        return out
    if cs is not None and bias_accumulate == accumulate:
        reduce_pair(slab, out, cs, bias_out, split, accumulate=accumulate)
    else:
        if cs is not None:
            reduce_into(cs, split, bias_out, accumulate=bias_accumulate)
        reduce_into(slab, split, out, accumulate)
    return out


def layerscale_wgrad(dsrc2d, a2d, w2, gamma, b2, *, dw2, dgamma, db2, compute_bf16=True, policy=None,
                     wgrad_target: int | None = None):
    """fc2 weight / bias / layer-scale gradients of out = x + gamma * (a W2^T + b2) from d_out:
    dW2 += gamma (.) d^T a, dgamma += rowdot(W2, d^T a) + b2 (.) colsum(d), db2 += gamma (.) colsum(d).
    The wgrad GEMM writes split-K slabs (+ colsum partials); ONE fused pass (a workgroup per row)
    reduces them and applies the layer-scale finish (sv_layerscale_wgrad_reduce) -- G = d^T a is
    never materialised."""
    M, C = dsrc2d.shape
    K4 = a2d.shape[1]
    split = _wgrad_split_for(C, K4, M, wgrad_target)
    cs = torch.empty(split * C, device=dsrc2d.device, dtype=torch.float32)
    if _bf16_slabs(C, K4, M, split, compute_bf16, policy):
        slab16 = torch.empty(split * C * K4, device=dsrc2d.device, dtype=torch.bfloat16)
        gemm(dsrc2d, a2d, M=C, N=K4, K=M, a_kmajor=False, b_kmajor=False, lda=C, ldb=K4, epilogue=nv.SV_EPI_SLAB,
             C=slab16, C2=cs, split_k=split, compute_bf16=True, policy=policy)
        _timed_call("fold", 2.0 * split * C * K4 + 8.0 * C * K4 + 4.0 * (split + 4) * C,
                    "sv_layerscale_wgrad_reduce_bf16", ptr(slab16), ptr(cs), split, ptr(w2), ptr(gamma), ptr(b2),
                    ptr(dw2), ptr(dgamma), ptr(db2), C, K4)
        return
    slab = torch.empty(split * C * K4, device=dsrc2d.device, dtype=torch.float32)
    G = torch.empty(C * K4, device=dsrc2d.device, dtype=torch.float32)
    if _fold_ok(split, C * K4, G, compute_bf16):
        # G = d^T a folded inside the wgrad GEMM; the finish then reads one G instead of `split` slabs
        gemm(dsrc2d, a2d, M=C, N=K4, K=M, a_kmajor=False, b_kmajor=False, lda=C, ldb=K4, epilogue=nv.SV_EPI_SLAB,
             C=slab, C2=cs, split_k=split, compute_bf16=compute_bf16, policy=policy,
             fold=(G, False, _fold_counters(dsrc2d.device, -(-C // 256) * -(-K4 // 256))))
        _timed_call("fold", 4.0 * (3 * C * K4 + (split + 4) * C), "sv_layerscale_wgrad_fold_finish", ptr(G), ptr(cs),
                    split, ptr(w2), ptr(gamma), ptr(b2), ptr(dw2), ptr(dgamma), ptr(db2), C, K4)
        return
    gemm(dsrc2d, a2d, M=C, N=K4, K=M, a_kmajor=False, b_kmajor=False, lda=C, ldb=K4, epilogue=nv.SV_EPI_SLAB,
         C=slab, C2=cs, split_k=split, compute_bf16=compute_bf16, policy=policy)
    _timed_call("fold", 4.0 * ((split + 2) * C * K4 + (split + 4) * C),
                "sv_layerscale_wgrad_reduce", ptr(slab), ptr(cs), split, ptr(w2), ptr(gamma), ptr(b2), ptr(dw2),
                ptr(dgamma), ptr(db2), None, C, K4)


# ----------------------------------------------------------------------------------------------
# reductions
def reduce_into(part: torch.Tensor, nparts: int, out: torch.Tensor, accumulate: bool = True, alpha: float = 1.0):
    """out (+)= alpha * sum of nparts partial rows -- one launch for any depth (sv_reduce_partials_pair)."""
    reduce_pair(part, out, None, None, nparts, accumulate=accumulate, alpha=alpha)


def reduce_pair(part_a: torch.Tensor, out_a: torch.Tensor, part_b: torch.Tensor | None, out_b: torch.Tensor | None,
                nparts: int, accumulate: bool = True, alpha: float = 1.0):
    """Two independent partial reductions with the same depth in ONE launch (weight + bias gradients)."""
    na = out_a.numel()
    _check(part_a.numel() >= nparts * na, "reduce_pair: partial buffer a too small")
    _check(out_a.dtype == torch.float32 and out_a.is_contiguous(), "reduce_pair: out must be contiguous f32")
    nb = 0
    if out_b is not None:
        nb = out_b.numel()
        _check(part_b is not None and part_b.numel() >= nparts * nb, "reduce_pair: partial buffer b too small")
        _check(out_b.dtype == torch.float32 and out_b.is_contiguous(), "reduce_pair: out must be contiguous f32")
    moved = 4.0 * (na + nb) * (nparts + 1 + int(bool(accumulate)))  # slabs read, out written (+ read)
    _timed_call("fold", moved, "sv_reduce_partials_pair", ptr(part_a), na, ptr(out_a), ptr(part_b), nb, ptr(out_b),
                nparts, float(alpha), int(accumulate))


def reduce_multi(segs: list, alpha: float = 1.0) -> None:
    """Independent partial reductions out (+)= alpha * sum_p part[p] in one launch per SV_MAX_RED_SEGS
    segments (sv_reduce_partials_multi).  segs: (part, out, P, accumulate) tuples, f32 contiguous."""
    for i in range(0, len(segs), nv.SV_MAX_RED_SEGS):
        chunk = segs[i:i + nv.SV_MAX_RED_SEGS]
        arr = (nv.RedSeg * len(chunk))()
        moved = 0.0
        for j, (part, out, P, acc) in enumerate(chunk):
            n = out.numel()
            _check(out.dtype == torch.float32 and out.is_contiguous() and part.numel() >= P * n,
                   "reduce_multi: bad segment")
            arr[j] = nv.RedSeg(ptr(part), ptr(out), n, int(P), int(bool(acc)))
            moved += 4.0 * n * (P + 1 + int(bool(acc)))
        _timed_call("fold", moved, "sv_reduce_partials_multi", arr, len(chunk), float(alpha))


def colsum_into(x2d: torch.Tensor, out: torch.Tensor, accumulate: bool = True):
    rows, C = x2d.shape
    P = value("sv_colsum_nparts", rows, C)
    part = torch.empty(P * C, device=x2d.device, dtype=torch.float32)
    call("sv_colsum", ptr(x2d), dt(x2d), rows, C, ptr(part))
    reduce_into(part, P, out, accumulate)


def colsum(x2d: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x2d.shape[1], device=x2d.device, dtype=torch.float32)
    colsum_into(x2d, out, accumulate=False)
    return out


# ----------------------------------------------------------------------------------------------
# LayerNorm
def layernorm_fwd(x2d, w, b, *, out_dtype, eps=EPS_LN):
    rows, C = x2d.shape
    y = torch.empty(rows, C, device=x2d.device, dtype=out_dtype)
    mean = torch.empty(rows, device=x2d.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    call("sv_layernorm_fwd", ptr(x2d), dt(x2d), ptr(w), ptr(b), ptr(y), dt(y), ptr(mean), ptr(rstd), rows, C, eps)
    return y, mean, rstd


def layernorm_bwd(dy2d, x2d, mean, rstd, w, *, dw, db, dx=None, accumulate_dx=False, out_dtype=torch.float32,
                  defer_reduce=False):
    """dx (+)= LayerNorm backward; dw/db (+)= the weight/bias gradient through per-block partials.
    ``defer_reduce``: return ``(dx, finish)`` instead, ``finish()`` folding the partials into dw/db on
    whatever stream is current when it is called (the ConvNeXt backward runs it on the weight-gradient
    side stream, off the data-gradient chain)."""
    rows, C = x2d.shape
    _check(tuple(dy2d.shape) == (rows, C) and dy2d.is_contiguous(), "layernorm_bwd: dy must be contiguous [rows,C]")
    if dx is None:
        dx = torch.empty(rows, C, device=x2d.device, dtype=out_dtype)
    P = value("sv_layernorm_bwd_nparts", rows, C)
    pw = torch.empty(2, P * C, device=x2d.device, dtype=torch.float32)
    # algorithmic: dy, x read; dx written (read too when accumulating); mean / rstd read
    nb = rows * C * (dy2d.element_size() + x2d.element_size() + dx.element_size() * (2 if accumulate_dx else 1)) + rows * 8
    _timed_call("ln_bwd", nb, "sv_layernorm_bwd", ptr(dy2d), dt(dy2d), ptr(x2d), dt(x2d), ptr(mean), ptr(rstd), ptr(w),
                ptr(dx), dt(dx), int(accumulate_dx), ptr(pw[0]), ptr(pw[1]), rows, C)
    if defer_reduce:
        def finish(record: bool = True, defer: list | None = None):
            if record:  # the caller may instead keep pw alive until the streams have joined
                pw.record_stream(torch.cuda.current_stream())
            if defer is not None:  # folded by the caller's reduce_multi launch
                defer += [(pw[0], dw, P, True), (pw[1], db, P, True)]
                return
            reduce_pair(pw[0], dw, pw[1], db, P)
        return dx, finish
    if dw is not None and db is not None:
        reduce_pair(pw[0], dw, pw[1], db, P)
    elif dw is not None:
        reduce_into(pw[0], P, dw)
    elif db is not None:
        reduce_into(pw[1], P, db)
    return dx


# ----------------------------------------------------------------------------------------------
# depthwise 7x7 + LN
# The depthwise conv on the matrix cores (csrc/dwmfma.hip, round 6): per channel a banded-Toeplitz GEMM along the image
# row on v_mfma_f32_16x16x32_bf16, with bf16 operands (the precision torch.autocast gives conv_dw).  Default: the bf16
# training forward (z kept) and the bf16-dz backward-data run on it (+1.3-1.4 % training step over the f32 VALU kernels,
# profiles/round6/r13g_*), and the tape-free eval forward (MFMA + LayerNorm beat the VALU one pass: S3 35.3 vs 44.5 us,
# r13l); SV_DW_MFMA=0 keeps the VALU kernels (dwconv.hip), which the f32 parity mode always uses.
DW_MFMA = os.environ.get("SV_DW_MFMA", "1") != "0"
# the weight gradient on the matrix cores (sv_dwconv7_bwd_weight_mfma): opt-in -- correct, but 20 % slower than the VALU
# ring kernel standalone and in the step (r13l: S3 39.0 vs 31.9 us; dw_wgrad 3.4-3.8 vs 2.9 ms/step)
DW_MFMA_WGRAD = DW_MFMA and os.environ.get("SV_DW_MFMA_WGRAD", "0") != "0"


def dwconv7_fwd_mfma(x4d, wdw, bdw):
    """z (bf16) = bf16(bdw + sum_tap bf16(w) bf16(x)) (sv_dwconv7_fwd_mfma)."""
    B, H, W, C = x4d.shape
    _check(C % 32 == 0 and x4d.is_contiguous() and x4d.dtype in (torch.float32, torch.bfloat16),
           "dwconv7_fwd_mfma: contiguous f32 / bf16 [B,H,W,C], C % 32 == 0")
    _check(wdw.dtype == torch.float32 and wdw.is_contiguous() and wdw.numel() == 49 * C and bdw.numel() == C,
           "dwconv7_fwd_mfma: f32 weight [C,1,7,7], bias [C]")
    z = torch.empty(B, H, W, C, device=x4d.device, dtype=torch.bfloat16)
    n = B * H * W * C
    _timed_call("dw_fwd", n * (x4d.element_size() + 2), "sv_dwconv7_fwd_mfma", ptr(x4d), dt(x4d), ptr(wdw), ptr(bdw),
                ptr(z), B, H, W, C, flops=98.0 * n)
    return z


def dwconv7_ln_fwd(x4d, wdw, bdw, lnw, lnb, *, act_dtype, eps=EPS_LN, save_z=True):
    """-> z (the conv output, saved for the LayerNorm backward; None when ``save_z`` is False and the one-pass form
    runs), y = LN(z), mean, rstd.  C = 128 / 256 / 512 over an f32 input run as ONE kernel (sv_dwconv7_ln_fused_ok),
    bitwise the two-launch result."""
    B, H, W, C = x4d.shape
    _check(C % 64 == 0, "dwconv7: C must be a multiple of 64")
    if DW_MFMA and act_dtype == torch.bfloat16:
        z = dwconv7_fwd_mfma(x4d, wdw, bdw)
        y, mean, rstd = layernorm_fwd(z.view(-1, C), lnw, lnb, out_dtype=act_dtype, eps=eps)
        return (z if save_z else None), y, mean, rstd
    act_code = SV_BF16 if act_dtype == torch.bfloat16 else SV_F32
    if not save_z and value("sv_dwconv7_ln_fused_ok", B, H, W, C, dt(x4d), act_code, act_code):
        z = None
    else:
        z = torch.empty(B, H, W, C, device=x4d.device, dtype=act_dtype)
    y = torch.empty(B * H * W, C, device=x4d.device, dtype=act_dtype)
    mean = torch.empty(B * H * W, device=x4d.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    n = B * H * W * C
    # algorithmic: x read once; z (saved for the LN backward) and y (the fc1 operand) written; mean / rstd
    nb = n * (x4d.element_size() + (z.element_size() if z is not None else 0) + y.element_size()) + B * H * W * 8
    _timed_call("dw_fwd", nb, "sv_dwconv7_ln_fwd", ptr(x4d), dt(x4d), ptr(wdw), ptr(bdw), ptr(lnw), ptr(lnb), eps, ptr(z),
                dt(y) if z is None else dt(z), ptr(y), dt(y), ptr(mean), ptr(rstd), B, H, W, C, fma=49.0 * n)
    return z, y, mean, rstd


def dwconv7_bwd_data(dz4d, wdw, dx4d, accumulate=True, dx_bf16=None):
    B, H, W, C = dz4d.shape
    _check(dx4d.shape == dz4d.shape and dx4d.dtype == torch.float32, "dwconv7_bwd_data: shape")
    if dx_bf16 is not None:
        _check(dx_bf16.numel() == dx4d.numel() and dx_bf16.dtype == torch.bfloat16, "dwconv7_bwd_data: bf16 copy")
    n = B * H * W * C
    # algorithmic: dz read; the f32 gradient stream dx written (and read when accumulating); its bf16 copy
    nb = n * (dz4d.element_size() + 4 * (2 if accumulate else 1) + (2 if dx_bf16 is not None else 0))
    if DW_MFMA and dz4d.dtype == torch.bfloat16 and C % 32 == 0:
        _timed_call("dw_bwd_data", nb, "sv_dwconv7_bwd_data_mfma", ptr(dz4d), ptr(wdw), ptr(dx4d), ptr(dx_bf16),
                    int(accumulate), B, H, W, C, flops=98.0 * n)
        return
    _timed_call("dw_bwd_data", nb, "sv_dwconv7_bwd_data", ptr(dz4d), dt(dz4d), ptr(wdw), ptr(dx4d), ptr(dx_bf16),
                int(accumulate), B, H, W, C, fma=49.0 * n)


def dwconv7_bwd_weight(dz4d, x4d, *, dw, db, defer: list | None = None):
    B, H, W, C = dz4d.shape
    mfma = DW_MFMA_WGRAD and dz4d.dtype == torch.bfloat16 and C % 16 == 0
    P = value("sv_dwconv7_bwd_weight_mfma_nparts" if mfma else "sv_dwconv7_bwd_weight_nparts", B, H, W, C)
    pw = torch.empty(P * C * 49, device=dz4d.device, dtype=torch.float32)
    pb = torch.empty(P * C, device=dz4d.device, dtype=torch.float32)
    # algorithmic: dz and x read once, the [C,49] + [C] gradient written (the partials are a design choice)
    nb = B * H * W * C * (dz4d.element_size() + x4d.element_size()) + C * 50 * 4
    if mfma:
        _timed_call("dw_wgrad", nb, "sv_dwconv7_bwd_weight_mfma", ptr(dz4d), ptr(x4d), dt(x4d), ptr(pw), ptr(pb),
                    B, H, W, C, flops=98.0 * B * H * W * C)
    else:
        _timed_call("dw_wgrad", nb, "sv_dwconv7_bwd_weight", ptr(dz4d), dt(dz4d), ptr(x4d), dt(x4d), ptr(pw), ptr(pb),
                    B, H, W, C, fma=49.0 * B * H * W * C)
    if defer is not None:
        defer += [(pw, dw, P, True), (pb, db, P, True)]
        return
    reduce_pair(pw, dw, pb, db, P)


# ----------------------------------------------------------------------------------------------
# stem / downsample / pool
def stem_fwd(img, w, b, lnw, lnb, *, eps=EPS_LN):
    B, Cin, H, W = img.shape
    _check(Cin == 3 and H % 4 == 0 and W % 4 == 0, "stem: expects [B,3,H,W] with H,W % 4 == 0")
    _check(img.dtype == torch.float32 and img.is_contiguous(), "stem: image must be contiguous f32 NCHW")
    C = w.shape[0]
    y = torch.empty(B, H // 4, W // 4, C, device=img.device, dtype=torch.float32)
    mean = torch.empty(B * (H // 4) * (W // 4), device=img.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    call("sv_stem_patchify_ln_fwd", ptr(img), ptr(w), ptr(b), ptr(lnw), ptr(lnb), eps, ptr(y), dt(y), ptr(mean),
         ptr(rstd), B, H, W, C)
    return y, mean, rstd


def stem_bwd(img, w, b, lnw, mean, rstd, dy, *, dw, db, dlnw, dlnb):
    B, _, H, W = img.shape
    C = w.shape[0]
    P = value("sv_stem_patchify_ln_bwd_nparts", B, H, W, C)
    pw = torch.empty(P * C * 48, device=img.device, dtype=torch.float32)
    pv = torch.empty(3, P * C, device=img.device, dtype=torch.float32)
    call("sv_stem_patchify_ln_bwd", ptr(img), ptr(w), ptr(b), ptr(lnw), ptr(mean), ptr(rstd), ptr(dy), ptr(pw),
         ptr(pv[0]), ptr(pv[1]), ptr(pv[2]), B, H, W, C)
    reduce_pair(pw, dw, pv[0], db, P)
    reduce_pair(pv[1], dlnw, pv[2], dlnb, P)


IMAGENET_MEAN = (0.485, 0.456, 0.406)  # torchvision Normalize constants of the reference transform
IMAGENET_STD = (0.229, 0.224, 0.225)


def _host3(v) -> ctypes.Array:
    return (ctypes.c_float * 3)(*[float(x) for x in v])


def stem_patchify(img, *, mean=IMAGENET_MEAN, std=IMAGENET_STD) -> torch.Tensor:
    """Stem patch rows for the MFMA stem conv: bf16 [B*(H/4)*(W/4), 64] (k = ci*16 + kh*4 + kw, 48..63
    zero).  img: the normalised f32 batch [B,3,H,W] or a uint8 grayscale batch [B,H,W] (the reference
    transform ToTensor + gray->RGB + Normalize(mean, std) is then applied in the gather)."""
    if img.dtype == torch.uint8:
        _check(img.dim() == 3 and img.is_contiguous(), "stem_patchify: uint8 input must be contiguous [B,H,W]")
        B, H, W = img.shape
        kind = nv.SV_IMG_U8_GRAY
    else:
        _check(img.dim() == 4 and img.shape[1] == 3 and img.dtype == torch.float32 and img.is_contiguous(),
               "stem_patchify: expects contiguous f32 [B,3,H,W]")
        B, _, H, W = img.shape
        kind = nv.SV_IMG_F32_NCHW
    _check(H % 4 == 0 and W % 4 == 0, "stem_patchify: H, W must be multiples of 4")
    patches = torch.empty(B * (H // 4) * (W // 4), 64, device=img.device, dtype=torch.bfloat16)
    call("sv_stem_patchify", ptr(img), kind, _host3(mean), _host3(std), ptr(patches), B, H, W)
    return patches


def stem_weight_pack(w) -> torch.Tensor:
    """timm stem.0.weight [C,3,4,4] f32 -> bf16 [C,64] (k 48..63 zero), the B operand of the stem GEMM."""
    C = w.shape[0]
    _check(w.numel() == C * 48 and w.dtype == torch.float32 and w.is_contiguous(), "stem_weight_pack: bad weight")
    out = torch.empty(C, 64, device=w.device, dtype=torch.bfloat16)
    call("sv_stem_weight_pack", ptr(w), ptr(out), C)
    return out


def normalize_u8_gray(img_u8, *, mean=IMAGENET_MEAN, std=IMAGENET_STD, out=None) -> torch.Tensor:
    """Device form of the reference transform tail (localization.py:196-233, 254): uint8 grayscale
    [B,H,W] -> convert("RGB") -> ToTensor (/255) -> Normalize(mean, std) -> f32 [B,3,H,W]."""
    _check(img_u8.dtype == torch.uint8 and img_u8.dim() == 3 and img_u8.is_contiguous(),
           "normalize_u8_gray: expects contiguous uint8 [B,H,W]")
    B, H, W = img_u8.shape
    _check((H * W) % 4 == 0, "normalize_u8_gray: H*W must be a multiple of 4")
    if out is None:
        out = torch.empty(B, 3, H, W, device=img_u8.device, dtype=torch.float32)
    _check(out.shape == (B, 3, H, W) and out.dtype == torch.float32 and out.is_contiguous(),
           "normalize_u8_gray: bad out")
    call("sv_normalize_u8_gray", ptr(img_u8), _host3(mean), _host3(std), ptr(out), B, H, W)
    return out


def augment_u8(img_u8: torch.Tensor, params: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Train-time flip / affine / colour jitter of decoded uint8 images on the device (row f1):
    ``img_u8`` [B,H,W] (grayscale) or [B,H,W,3] (RGB), ``params`` float64 [B,10] from
    ``training.datasets.augment.sample_params`` (torchvision's draws).  Bitwise equal to the PIL
    operations torchvision applies on the host (sv_augment_u8)."""
    _check(img_u8.dtype == torch.uint8 and img_u8.is_contiguous() and img_u8.dim() in (3, 4),
           "augment_u8: expects contiguous uint8 [B,H,W] or [B,H,W,3]")
    B, H, W = img_u8.shape[:3]
    C = 1 if img_u8.dim() == 3 else img_u8.shape[3]
    _check(C in (1, 3), "augment_u8: 1 or 3 channels")
    params = params.to(device=img_u8.device, dtype=torch.float64).contiguous()
    _check(tuple(params.shape) == (B, 10), "augment_u8: params must be [B,10]")
    if out is None:
        out = torch.empty_like(img_u8)
    _check(out.shape == img_u8.shape and out.dtype == torch.uint8 and out.is_contiguous()
           and out.data_ptr() != img_u8.data_ptr(), "augment_u8: bad out")
    rows = torch.empty(B * H, device=img_u8.device, dtype=torch.int32)
    call("sv_augment_u8", ptr(img_u8), ptr(out), B, H, W, C, ptr(params), ptr(rows))
    return out


def resize_u8(src: torch.Tensor, desc: torch.Tensor, coef: torch.Tensor, B: int, H: int, W: int, C: int,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """PIL Image.resize((W, H), BILINEAR) of a ragged uint8 batch on the device (row f1, sv_resize_u8):
    ``src`` flat uint8, ``desc`` int64 [B,8] and ``coef`` int32 tables from
    ``training.datasets.resize.ragged_batch``.  Returns uint8 [B,H,W] (C = 1) or [B,H,W,3]."""
    _check(src.dtype == torch.uint8 and src.is_contiguous(), "resize_u8: src must be contiguous uint8")
    _check(desc.dtype == torch.int64 and tuple(desc.shape) == (B, 8) and desc.is_contiguous(), "resize_u8: desc [B,8]")
    _check(coef.dtype == torch.int32 and coef.is_contiguous(), "resize_u8: coef must be int32")
    _check(C in (1, 3), "resize_u8: C must be 1 or 3")
    shape = (B, H, W) if C == 1 else (B, H, W, 3)
    if out is None:
        out = torch.empty(shape, device=src.device, dtype=torch.uint8)
    _check(tuple(out.shape) == shape and out.dtype == torch.uint8 and out.is_contiguous(), "resize_u8: bad out")
    call("sv_resize_u8", ptr(src), ptr(desc), ptr(coef), B, H, W, C, ptr(out))
    return out


def device_images(batch: dict, device) -> torch.Tensor:
    """The decoded uint8 image batch of a device_transform loader on ``device``, resized (ragged batch:
    "resize" = ragged_batch(...)) and augmented ("augment") there -- the reference's Resize -> [flip /
    affine / jitter] on the GPU; ToTensor -> Normalize then run inside the backbone's stem gather."""
    rz = batch.get("resize")
    if rz is not None:
        H, W, C = (int(v) for v in rz["out_hw"])
        img = resize_u8(rz["src"].to(device, non_blocking=True), rz["desc"].to(device, non_blocking=True),
                        rz["coef"].to(device, non_blocking=True), rz["desc"].shape[0], H, W, C)
    else:
        img = batch["image"].to(device, non_blocking=True)
    if "augment" in batch:
        img = augment_u8(img, batch["augment"].to(device, non_blocking=True))
    return img


def downsample_fwd(x4d, lnw, lnb, *, act_dtype, eps=EPS_LN):
    B, H, W, C = x4d.shape
    _check(H % 2 == 0 and W % 2 == 0, "downsample: H, W must be even")
    patches = torch.empty(B * (H // 2) * (W // 2), 4 * C, device=x4d.device, dtype=act_dtype)
    mean = torch.empty(B * H * W, device=x4d.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    call("sv_downsample_ln_patch2_fwd", ptr(x4d), ptr(lnw), ptr(lnb), eps, ptr(patches), dt(patches), ptr(mean),
         ptr(rstd), B, H, W, C)
    return patches, mean, rstd


def downsample_bwd(dpatches, x4d, mean, rstd, lnw, *, dlnw, dlnb, with_bf16=False):
    """-> dx (f32 [B,H,W,C]) and, with ``with_bf16``, its bf16 GEMM-operand copy (else None)."""
    B, H, W, C = x4d.shape
    dx = torch.empty(B, H, W, C, device=x4d.device, dtype=torch.float32)
    dxb = torch.empty(B, H, W, C, device=x4d.device, dtype=torch.bfloat16) if with_bf16 else None
    P = value("sv_downsample_ln_patch2_bwd_nparts", B, H, W, C)
    pv = torch.empty(2, P * C, device=x4d.device, dtype=torch.float32)
    call("sv_downsample_ln_patch2_bwd", ptr(dpatches), ptr(x4d), ptr(mean), ptr(rstd), ptr(lnw), ptr(dx), ptr(dxb),
         ptr(pv[0]), ptr(pv[1]), B, H, W, C)
    reduce_pair(pv[0], dlnw, pv[1], dlnb, P)
    return dx, dxb


def pool_ln_fwd(x4d, lnw, lnb, *, eps=EPS_LN):
    B, H, W, C = x4d.shape
    pooled = torch.empty(B, C, device=x4d.device, dtype=torch.float32)
    feat = torch.empty_like(pooled)
    mean = torch.empty(B, device=x4d.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    call("sv_pool_ln_fwd", ptr(x4d), ptr(lnw), ptr(lnb), eps, ptr(pooled), ptr(feat), ptr(mean), ptr(rstd), B,
         H * W, C)
    return feat, pooled, mean, rstd


def pool_ln_bwd(dfeat, pooled, mean, rstd, lnw, shape, *, dlnw, dlnb, with_bf16=False):
    """-> dx (f32 [B,H,W,C]) and, with ``with_bf16``, its bf16 GEMM-operand copy (else None)."""
    B, H, W, C = shape
    dx = torch.empty(B, H, W, C, device=dfeat.device, dtype=torch.float32)
    dxb = torch.empty(B, H, W, C, device=dfeat.device, dtype=torch.bfloat16) if with_bf16 else None
    pv = torch.empty(2, B * C, device=dfeat.device, dtype=torch.float32)
    call("sv_pool_ln_bwd", ptr(dfeat.contiguous()), ptr(pooled), ptr(mean), ptr(rstd), ptr(lnw), ptr(dx), ptr(dxb),
         ptr(pv[0]), ptr(pv[1]), B, H * W, C)
    reduce_pair(pv[0], dlnw, pv[1], dlnb, B)
    return dx, dxb


# ----------------------------------------------------------------------------------------------
# optimizer pieces
def scale_rows_bf16(W: torch.Tensor, scale: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """bf16(W * scale[:, None]) for a 2-D f32 weight (fc2 weight with the layer scale folded in)."""
    rows, cols = W.shape
    _check(W.dtype == torch.float32 and W.is_contiguous() and scale.numel() == rows, "scale_rows_bf16: bad args")
    if out is None:
        out = torch.empty(rows, cols, device=W.device, dtype=torch.bfloat16)
    _check(out.shape == (rows, cols) and out.dtype == torch.bfloat16 and out.is_contiguous(), "scale_rows_bf16: bad out")
    call("sv_scale_rows_bf16", ptr(W), ptr(scale), ptr(out), rows, cols)
    return out


def cast_bf16(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _check(x.dtype == torch.float32 and x.is_contiguous(), "cast_bf16: need contiguous f32")
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
    call("sv_cast_f32_bf16", ptr(x), ptr(out), x.numel())
    return out


def grad_clip_coef(g_flat: torch.Tensor, max_norm: float) -> torch.Tensor:
    """Device tensor [norm, coef] with coef = min(1, max_norm/(norm+1e-6)) -- no host sync."""
    n = g_flat.numel()
    P = value("sv_sqnorm_nparts", n)
    part = torch.empty(P, device=g_flat.device, dtype=torch.float32)
    call("sv_sqnorm_partial", ptr(g_flat), n, ptr(part))
    out = torch.empty(2, device=g_flat.device, dtype=torch.float32)
    call("sv_clip_coef", ptr(part), P, float(max_norm), ptr(out))
    return out


def adamw_hyper(lr: float, beta1: float, beta2: float, step: int) -> list[float]:
    """[lr, 1 - b1^step, sqrt(1 - b2^step)] as f32 values, rounded exactly as sv_adamw_flat derives
    them on the host (double power, f32 rounding, f32 sqrt) -- the device operand of adamw_flat(hyper=)."""
    b1, b2 = float(np.float32(beta1)), float(np.float32(beta2))  # the C ABI takes the betas as f32
    bc1 = np.float32(1.0 - b1 ** step)
    bc2 = np.float32(1.0 - b2 ** step)
    return [float(np.float32(lr)), float(bc1), float(np.sqrt(bc2, dtype=np.float32))]


def adamw_flat(p, g, m, v, p_bf16, *, lr, beta1, beta2, eps, weight_decay, step, grad_scale=None, hyper=None):
    """``hyper``: optional f32 device tensor [3] (adamw_hyper) replacing lr/step -- graph replay."""
    n = p.numel()
    _check(g.numel() == n and m.numel() == n and v.numel() == n, "adamw_flat: size mismatch")
    if hyper is not None:
        _check(hyper.dtype == torch.float32 and hyper.is_cuda and hyper.numel() >= 3, "adamw_flat: hyper")
        call("sv_adamw_flat_dev", ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), n, float(beta1), float(beta2),
             float(eps), float(weight_decay), ptr(hyper), ptr(grad_scale))
        return
    # algorithmic: p, g, m, v read; p, m, v written; the bf16 shadow written (30 B / parameter)
    nb = n * (28 + (2 if p_bf16 is not None else 0))
    _timed_call("adamw", nb, "sv_adamw_flat", ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), n, float(lr), float(beta1),
                float(beta2), float(eps), float(weight_decay), int(step), ptr(grad_scale))


# ----------------------------------------------------------------------------------------------
# ResNet-18/50: implicit-GEMM convolution, BatchNorm (train-mode batch statistics), pooling
EPS_BN = 1e-5


def _is_pow2(v: int) -> bool:
    return v > 0 and (v & (v - 1)) == 0


def conv_out_hw(H: int, W: int, k: int, stride: int, pad: int) -> tuple[int, int]:
    return (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1


def conv_shape(B, H, W, Cs, Cout, k, stride, pad, Cin=None) -> nv.ConvShape:
    s = nv.ConvShape()
    s.B, s.H, s.W, s.Cs, s.Cout = B, H, W, Cs, Cout
    s.KH = s.KW = k
    s.stride, s.pad = stride, pad
    s.Cin = Cs if Cin is None else Cin
    _check(_is_pow2(Cs) and Cs >= 4 and Cout % 8 == 0 and 0 < s.Cin <= Cs and stride in (1, 2),
           f"conv: unsupported shape Cs={Cs} Cout={Cout} Cin={s.Cin} stride={stride}")
    return s


def conv_weight_pack(w: torch.Tensor, Cs: int, dtype: torch.dtype) -> torch.Tensor:
    """torch weight [Cout][Cin][k][k] f32 -> packed [Cout][k*k][Cs] (`dtype`), channels >= Cin zero."""
    Cout, Cin, KH, KW = w.shape
    _check(w.dtype == torch.float32 and w.is_contiguous() and KH == KW, "conv_weight_pack: need contiguous f32 [Co,Ci,k,k]")
    s = conv_shape(1, KH, KW, Cs, Cout, KH, 1, 0, Cin)
    wp = torch.empty(Cout, KH * KW, Cs, device=w.device, dtype=dtype)
    call("sv_conv_weight_pack", ptr(w), ptr(wp), dt(wp), ctypes.byref(s))
    return wp


def conv_weight_pack_multi(items: list, dtype: torch.dtype) -> list:
    """conv_weight_pack for several weights in one launch per SV_MAX_PACK_SEGS (sv_conv_weight_pack_multi).
    items: (w f32 [Cout][Cin][k][k], Cs) pairs -> the packed [Cout][k*k][Cs] tensors, in order."""
    out = []
    for i in range(0, len(items), nv.SV_MAX_PACK_SEGS):
        chunk = items[i:i + nv.SV_MAX_PACK_SEGS]
        segs = (nv.PackSeg * len(chunk))()
        for j, (w, Cs) in enumerate(chunk):
            Cout, Cin, KH, KW = w.shape
            _check(w.dtype == torch.float32 and w.is_contiguous() and KH == KW and Cs >= Cin,
                   "conv_weight_pack_multi: need contiguous f32 [Co,Ci,k,k] and Cs >= Ci")
            wp = torch.empty(Cout, KH * KW, Cs, device=w.device, dtype=dtype)
            segs[j] = nv.PackSeg(ptr(w), ptr(wp), Cout, Cin, KH * KW, Cs)
            out.append(wp)
        call("sv_conv_weight_pack_multi", segs, len(chunk), SV_BF16 if dtype == torch.bfloat16 else SV_F32)
    return out


def _conv_check_x(x: torch.Tensor, s: nv.ConvShape, dtype: torch.dtype, who: str) -> None:
    _check(x.is_contiguous() and tuple(x.shape) == (s.B, s.H, s.W, s.Cs) and x.dtype == dtype,
           f"{who}: x must be contiguous {dtype} [B,H,W,Cs]={(s.B, s.H, s.W, s.Cs)}, got {tuple(x.shape)} {x.dtype}")


def _pointwise(s: nv.ConvShape, dtype: torch.dtype) -> bool:
    """1x1 / stride 1 / no padding over unpadded channels in bf16: in NHWC the conv IS a GEMM over
    [B*H*W, C] rows, so it runs on the LDS-DMA MFMA GEMM (sv_gemm v3) instead of the implicit-GEMM
    conv kernel (ResNet-50 bottleneck conv1 / conv3: ~half of its conv FLOPs)."""
    return (s.KH == 1 and s.KW == 1 and s.stride == 1 and s.pad == 0 and s.Cs == s.Cin and dtype == torch.bfloat16
            and s.Cs % 32 == 0 and s.Cout % 32 == 0)


# gathered forward convolutions split K only from this many 32-deep k-steps (round 4, profiles/round4/
# r8e_conv_split_sweep.txt: layer2's 3x3 forward, K = 1152, 128 tiles, runs in 30 us unsplit against 35 + a 7 us
# finish at split 2; layer3 / 4, K = 2304 / 4608, are fastest at split 4 / 8 as before)
_CONV_FWD_MIN_KSTEPS = int(os.environ.get("SV_CONV_FWD_MIN_KSTEPS", "64"))


def _conv_split(M: int, N: int, K: int, min_ksteps: int = 32) -> int:
    """split-K depth of a bf16 conv GEMM whose grid of 256x128 tiles would not give every CU a workgroup
    (ResNet layer3/4 at 256 px: 32-128 tiles, each a long latency-bound chain of 32-deep k-steps):
    about one workgroup per CU, >= 16 k-steps per slice, <= 32 MiB of f32 slabs (written by the GEMM,
    read back by sv_gemm_slab_finish), at most 16 slices.  1 = no split (also below ``min_ksteps`` k-steps, where
    the slab round trip costs more than the chain it shortens)."""
    tiles = -(-M // 256) * -(-N // 128)
    ksteps = K // 32
    if tiles >= 192 or ksteps < min_ksteps:
        return 1
    return max(1, min(-(-256 // tiles), ksteps // 16, (32 << 20) // (M * N * 4), 16))


def _gathered(s: nv.ConvShape, dtype: torch.dtype) -> bool:
    """the bf16 gathered-operand GEMM path of sv_conv_fwd (csrc/conv.hip conv_fwd_impl)"""
    return dtype == torch.bfloat16 and s.Cs >= 32 and _is_pow2(s.Cs) and (s.KH * s.KW * s.Cs) % 32 == 0


def _stem8(s: nv.ConvShape, dtype: torch.dtype) -> bool:
    """the bf16 8-channel gathered path of sv_conv_fwd (conv.hip mode 6: the ResNet stem over its zero-padded
    RGB operand, one tap per 16-B chunk)"""
    return (_STEM_GATHER and dtype == torch.bfloat16 and s.Cs == 8 and s.KH == s.KW and s.KH <= 7
            and s.Cout % 8 == 0)


# SV_STEM_GATHER=0: the stem forward on the register-staged conv kernel plus a BatchNorm statistics pass (A/B runs)
_STEM_GATHER = os.environ.get("SV_STEM_GATHER", "1") != "0"


def _slab_finish(work: torch.Tensor, split: int, M: int, N: int, C: torch.Tensor, *, accumulate: bool = False,
                 stats: torch.Tensor | None = None) -> None:
    _timed_call("fold", 4.0 * M * N * (split + 1 + int(bool(accumulate))), "sv_gemm_slab_finish", ptr(work), split, M,
                N, ptr(C), dt(C), N, int(accumulate), ptr(stats))


def _pointwise_fwd(x, wp, s, y, M, stats=None, policy=None):
    """1x1 conv forward as a GEMM over [M, Cs] rows; split-K + slab finish when the grid is small."""
    split = _conv_split(M, s.Cout, s.Cs)
    if split > 1:
        work = torch.empty(split * M * s.Cout, device=x.device, dtype=torch.float32)
        gemm(x.view(M, s.Cs), wp.view(s.Cout, s.Cs), M=M, N=s.Cout, K=s.Cs, a_kmajor=True, b_kmajor=True, lda=s.Cs,
             ldb=s.Cs, C=work, epilogue=nv.SV_EPI_SLAB, split_k=split, compute_bf16=True, policy=policy)
        _slab_finish(work, split, M, s.Cout, y, stats=stats)
    elif stats is not None:
        gemm(x.view(M, s.Cs), wp.view(s.Cout, s.Cs), M=M, N=s.Cout, K=s.Cs, a_kmajor=True, b_kmajor=True, lda=s.Cs,
             ldb=s.Cs, C=y.view(M, s.Cout), C2=stats, epilogue=nv.SV_EPI_STORE_STATS, compute_bf16=True,
             policy=policy)
    else:
        gemm(x.view(M, s.Cs), wp.view(s.Cout, s.Cs), M=M, N=s.Cout, K=s.Cs, a_kmajor=True, b_kmajor=True, lda=s.Cs,
             ldb=s.Cs, C=y.view(M, s.Cout), compute_bf16=True, policy=policy)


def conv_fwd(x: torch.Tensor, wp: torch.Tensor, s: nv.ConvShape, out_dtype: torch.dtype,
             policy: "nv.GemmPolicy | None" = None) -> torch.Tensor:
    _conv_check_x(x, s, wp.dtype, "conv_fwd")
    _check(tuple(wp.shape) == (s.Cout, s.KH * s.KW, s.Cs), "conv_fwd: packed weight shape")
    OH, OW = conv_out_hw(s.H, s.W, s.KH, s.stride, s.pad)
    y = torch.empty(s.B, OH, OW, s.Cout, device=x.device, dtype=out_dtype)
    if _pointwise(s, wp.dtype):
        _pointwise_fwd(x, wp, s, y, s.B * s.H * s.W, policy=policy)
        return y
    M, K = s.B * OH * OW, s.KH * s.KW * s.Cs
    split = _conv_split(M, s.Cout, K, _CONV_FWD_MIN_KSTEPS) if _gathered(s, wp.dtype) else 1
    if split > 1:
        work = torch.empty(split * M * s.Cout, device=x.device, dtype=torch.float32)
        call("sv_conv_fwd_split", ptr(x), ptr(wp), ptr(y), dt(y), dt(wp), ctypes.byref(s), None, ptr(work), split,
             nv.pol_ref(policy))
        return y
    call("sv_conv_fwd", ptr(x), ptr(wp), ptr(y), dt(y), dt(wp), ctypes.byref(s), nv.pol_ref(policy))
    return y


_ONES: dict = {}


def _ones(n: int, device: torch.device) -> torch.Tensor:
    """Cached f32 ones[n] per device (the gamma of an in-place accumulate epilogue): no fill launch per call."""
    key = (n, device)
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(n, device=device, dtype=torch.float32)
    return t


def conv_fwd_bn_stats(x: torch.Tensor, wp: torch.Tensor, s: nv.ConvShape, out_dtype: torch.dtype,
                      policy: "nv.GemmPolicy | None" = None):
    """conv_fwd plus the train-mode BatchNorm statistics of y straight from the GEMM epilogue
    (SV_EPI_STORE_STATS: no separate read pass over y) -> (y, partials [ceil(M/64)][2][Cout] f32), or
    (y, None) when the conv runs on a path without that epilogue (then use bn_stats(y))."""
    if wp.dtype != torch.bfloat16 or out_dtype != torch.bfloat16 or s.Cout % 8:
        return conv_fwd(x, wp, s, out_dtype, policy), None
    OH, OW = conv_out_hw(s.H, s.W, s.KH, s.stride, s.pad)
    M = s.B * OH * OW
    if _pointwise(s, wp.dtype):
        if s.Cs % 32:
            return conv_fwd(x, wp, s, out_dtype, policy), None
        _conv_check_x(x, s, wp.dtype, "conv_fwd")
        y = torch.empty(s.B, OH, OW, s.Cout, device=x.device, dtype=out_dtype)
        part = torch.empty((M + 63) // 64, 2, s.Cout, device=x.device, dtype=torch.float32)
        _pointwise_fwd(x, wp, s, y, M, stats=part, policy=policy)
        return y, part
    if not (_gathered(s, wp.dtype) or _stem8(s, wp.dtype)):
        return conv_fwd(x, wp, s, out_dtype, policy), None
    _conv_check_x(x, s, wp.dtype, "conv_fwd")
    _check(tuple(wp.shape) == (s.Cout, s.KH * s.KW, s.Cs), "conv_fwd: packed weight shape")
    y = torch.empty(s.B, OH, OW, s.Cout, device=x.device, dtype=out_dtype)
    part = torch.empty((M + 63) // 64, 2, s.Cout, device=x.device, dtype=torch.float32)
    split = 1 if _stem8(s, wp.dtype) else _conv_split(M, s.Cout, s.KH * s.KW * s.Cs, _CONV_FWD_MIN_KSTEPS)
    if split > 1:
        work = torch.empty(split * M * s.Cout, device=x.device, dtype=torch.float32)
        call("sv_conv_fwd_split", ptr(x), ptr(wp), ptr(y), dt(y), dt(wp), ctypes.byref(s), ptr(part), ptr(work), split,
             nv.pol_ref(policy))
    else:
        call("sv_conv_fwd_stats", ptr(x), ptr(wp), ptr(y), dt(y), dt(wp), ctypes.byref(s), ptr(part), nv.pol_ref(policy))
    return y, part


def bn_stats_from_partials(part: torch.Tensor, rows: int, *, eps: float = EPS_BN, momentum: float = 0.1,
                           running_mean=None, running_var=None, num_batches_tracked=None):
    """(mean, rstd) from conv_fwd_bn_stats' unshifted partials; running stats updated like bn_stats."""
    P, two, C = part.shape
    _check(two == 2 and part.dtype == torch.float32 and part.is_contiguous(), "bn_stats_from_partials: bad partials")
    mean = torch.empty(C, device=part.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    _fin("sv_bn_stats_finish", None, SV_F32, ptr(part), P, rows, C, float(eps), float(momentum), ptr(mean),
         ptr(rstd), ptr(running_mean), ptr(running_var), ptr(num_batches_tracked), *_fin_ws(part.device))
    return mean, rstd


def conv_bwd_data(dy: torch.Tensor, wp: torch.Tensor, s: nv.ConvShape, *, dx: torch.Tensor | None = None,
                  accumulate: bool = False, dx_dtype: torch.dtype = torch.float32,
                  policy: "nv.GemmPolicy | None" = None) -> torch.Tensor:
    OH, OW = conv_out_hw(s.H, s.W, s.KH, s.stride, s.pad)
    _check(dy.is_contiguous() and tuple(dy.shape) == (s.B, OH, OW, s.Cout) and dy.dtype == wp.dtype,
           "conv_bwd_data: dy must be contiguous [B,OH,OW,Cout] in the compute dtype")
    _check(_is_pow2(s.Cout), "conv_bwd_data: Cout must be a power of two")
    if dx is None:
        _check(not accumulate, "conv_bwd_data: accumulate needs dx")
        dx = torch.empty(s.B, s.H, s.W, s.Cs, device=dy.device, dtype=dx_dtype)
    _check(dx.is_contiguous() and tuple(dx.shape) == (s.B, s.H, s.W, s.Cs), "conv_bwd_data: dx shape")
    if _pointwise(s, wp.dtype) and (not accumulate or dx.dtype == torch.float32):
        M = s.B * s.H * s.W
        split = _conv_split(M, s.Cs, s.Cout)
        if split > 1:
            work = torch.empty(split * M * s.Cs, device=dy.device, dtype=torch.float32)
            gemm(dy.view(M, s.Cout), wp.view(s.Cout, s.Cs), M=M, N=s.Cs, K=s.Cout, a_kmajor=True, b_kmajor=False,
                 lda=s.Cout, ldb=s.Cs, C=work, epilogue=nv.SV_EPI_SLAB, split_k=split, compute_bf16=True, policy=policy)
            _slab_finish(work, split, M, s.Cs, dx, accumulate=accumulate)
        elif accumulate:  # dx += dy W: the layer-scale/residual epilogue with gamma = 1, residual = dx (in place)
            ones = _ones(s.Cs, dy.device)
            gemm(dy.view(M, s.Cout), wp.view(s.Cout, s.Cs), M=M, N=s.Cs, K=s.Cout, a_kmajor=True, b_kmajor=False,
                 lda=s.Cout, ldb=s.Cs, C=dx.view(M, s.Cs), epilogue=nv.SV_EPI_BIAS_GAMMA_RES, gamma=ones,
                 aux=dx.view(M, s.Cs), compute_bf16=True, policy=policy)
        else:
            gemm(dy.view(M, s.Cout), wp.view(s.Cout, s.Cs), M=M, N=s.Cs, K=s.Cout, a_kmajor=True, b_kmajor=False,
                 lda=s.Cout, ldb=s.Cs, C=dx.view(M, s.Cs), compute_bf16=True, policy=policy)
        return dx
    T = s.KH * s.KW
    # (a bf16 dx accumulates here too -- the ResNet gradient stream: the sum in f32, stored bf16 -- rather than in
    # the pointwise path above, whose residual epilogue reads an f32 operand)
    if (wp.dtype == torch.bfloat16 and s.stride == 1 and s.Cout >= 32 and s.Cs % 8 == 0 and (T * s.Cout) % 32 == 0):
        M = s.B * s.H * s.W
        split = _conv_split(M, s.Cs, T * s.Cout)
        if split > 1:
            work = torch.empty(split * M * s.Cs, device=dy.device, dtype=torch.float32)
            call("sv_conv_bwd_data_split", ptr(dy), ptr(wp), ptr(dx), dt(dx), int(accumulate), dt(wp),
                 ctypes.byref(s), ptr(work), split, nv.pol_ref(policy))
            return dx
    if wp.dtype == torch.bfloat16 and s.stride == 2 and s.Cout >= 32 and s.Cs % 8 == 0:
        # stride 2: one gathered GEMM per output parity class into compact f32 slabs + one scatter pass
        # (csrc/conv.hip dgrad_s2_scatter_kernel); the workspace holds every class's slabs.  Even H, W
        # without a split: the one-launch form stores each class's rows straight into dx (no workspace)
        M = s.B * s.H * s.W
        split = _s2_split(s, M, T)
        if split == 1 and _s2_direct(s):
            call("sv_conv_bwd_data", ptr(dy), ptr(wp), ptr(dx), dt(dx), int(accumulate), dt(wp), ctypes.byref(s),
                 nv.pol_ref(policy))
            return dx
        work = torch.empty(split * M * s.Cs, device=dy.device, dtype=torch.float32)
        call("sv_conv_bwd_data_split", ptr(dy), ptr(wp), ptr(dx), dt(dx), int(accumulate), dt(wp),
             ctypes.byref(s), ptr(work), split, nv.pol_ref(policy))
        return dx
    call("sv_conv_bwd_data", ptr(dy), ptr(wp), ptr(dx), dt(dx), int(accumulate), dt(wp), ctypes.byref(s),
         nv.pol_ref(policy))
    return dx


# stride-2 data gradients stored straight into dx by the parity-class GEMM's epilogue (csrc/gemm3.hip mode 5
# with remapped rows); 0 = the compact f32 slabs + scatter pass (A/B and the bitwise cross-check)
_S2_DIRECT = os.environ.get("SV_S2_DIRECT", "1") != "0"
# no split-K for the stride-2 dgrads that the one-launch form takes: the four classes already give the grid
# 4x the tiles, and the split's slabs cost more than the longer chains (+0.6 %, r9j); SV_S2_NOSPLIT=0 restores it
_S2_NOSPLIT = os.environ.get("SV_S2_NOSPLIT", "1") != "0"


def _s2_direct(s: nv.ConvShape) -> bool:
    return _S2_DIRECT and s.stride == 2 and s.H % 2 == 0 and s.W % 2 == 0


def _s2_split(s: nv.ConvShape, M: int, T: int) -> int:
    """split-K depth of a stride-2 dgrad's per-class GEMMs (M = B*H*W dx pixels, T taps)"""
    if _S2_NOSPLIT and _s2_direct(s):
        return 1
    return _conv_split(M // 4, s.Cs, max(32, (T * s.Cout) // 4))


def _al16(*ts) -> bool:
    return all(t.data_ptr() % 16 == 0 for t in ts)


def conv_bwd_data_bn(dy: torch.Tensor, wp: torch.Tensor, s: nv.ConvShape, y: torch.Tensor, mean: torch.Tensor,
                     rstd: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, *, unsplit: bool = True,
                     policy: "nv.GemmPolicy | None" = None):
    """conv_bwd_data (bf16 dx, no accumulate) fused with the backward statistics of the BatchNorm + ReLU that
    produced the conv's input: y [B,H,W,Cs] is that BatchNorm's input (bf16), mean / rstd its batch statistics,
    gamma / beta its affine parameters.  -> (dx, part), part = f32 [ceil(B*H*W/64)][2][Cs] partial sums of g
    and g*xhat (g = dx * relu mask) for bn_bwd(part=...), summed by the GEMM epilogue (SV_EPI_STORE_BN_BWD)
    or, for split-K shapes, by the finish that reads the slabs anyway (sv_gemm_slab_finish_bn_bwd): no
    statistics pass over dx and y.  ``unsplit=False`` fuses the split-K shapes only.  Stride 2 (even H, W,
    no split): the one-launch parity-class GEMM with the same epilogue, 4 * ceil(B*H*W/256) partial rows
    (one run per class).  None when the shape is not on these paths (odd stride-2 grids, split stride-2
    shapes, fp32, unaligned parameters): use conv_bwd_data + bn_bwd."""
    if wp.dtype != torch.bfloat16 or y.dtype != torch.bfloat16 or s.Cs % 8 or s.stride not in (1, 2):
        return None
    M = s.B * s.H * s.W
    T = s.KH * s.KW
    pw = _pointwise(s, wp.dtype)
    s2 = s.stride == 2
    if s2:  # the one-launch parity-class GEMM without a split; partials [4][ceil(M/4/64)][2][Cs]
        if not (_s2_direct(s) and T > 1 and _is_pow2(s.Cout) and s.Cout >= 32
                and _s2_split(s, M, T) == 1):
            return None
        split = 1
    elif pw:
        split = _conv_split(M, s.Cs, s.Cout)
    elif _is_pow2(s.Cout) and s.Cout >= 32 and (T * s.Cout) % 32 == 0:
        split = _conv_split(M, s.Cs, T * s.Cout)
    else:
        return None
    if split < 2 and not unsplit:
        return None
    OH, OW = conv_out_hw(s.H, s.W, s.KH, s.stride, s.pad)
    _check(dy.is_contiguous() and tuple(dy.shape) == (s.B, OH, OW, s.Cout) and dy.dtype == wp.dtype,
           "conv_bwd_data_bn: dy must be contiguous [B,OH,OW,Cout] bf16")
    _check(y.is_contiguous() and y.numel() == M * s.Cs, "conv_bwd_data_bn: y shape")
    prm = [p_.detach() for p_ in (mean, rstd, gamma, beta)]
    if not _al16(y, *prm) or any(p_.dtype != torch.float32 or not p_.is_contiguous() for p_ in prm):
        return None
    ref = nv.BnRef(ptr(prm[0]), ptr(prm[1]), ptr(prm[2]), ptr(prm[3]))
    dx = torch.empty(s.B, s.H, s.W, s.Cs, device=dy.device, dtype=torch.bfloat16)
    prows = 4 * ((M // 4 + 63) // 64) if s2 else (M + 63) // 64
    part = torch.empty(prows, 2, s.Cs, device=dy.device, dtype=torch.float32)
    work = torch.empty(split * M * s.Cs, device=dy.device, dtype=torch.float32) if split > 1 else None
    if pw and split > 1:
        gemm(dy.view(M, s.Cout), wp.view(s.Cout, s.Cs), M=M, N=s.Cs, K=s.Cout, a_kmajor=True, b_kmajor=False,
             lda=s.Cout, ldb=s.Cs, C=work, epilogue=nv.SV_EPI_SLAB, split_k=split, compute_bf16=True, policy=policy)
        call("sv_gemm_slab_finish_bn_bwd", ptr(work), split, M, s.Cs, ptr(dx), ptr(y), ctypes.byref(ref), ptr(part))
    elif pw:
        gemm(dy.view(M, s.Cout), wp.view(s.Cout, s.Cs), M=M, N=s.Cs, K=s.Cout, a_kmajor=True, b_kmajor=False,
             lda=s.Cout, ldb=s.Cs, C=dx.view(M, s.Cs), C2=part, epilogue=nv.SV_EPI_STORE_BN_BWD,
             aux=y.view(M, s.Cs), compute_bf16=True, bn=ref, policy=policy)
    else:
        call("sv_conv_bwd_data_bn", ptr(dy), ptr(wp), ptr(dx), dt(wp), ctypes.byref(s), ptr(y), ctypes.byref(ref),
             ptr(part), ptr(work), split, nv.pol_ref(policy))
    return dx, part


def conv_bwd_weight(dy: torch.Tensor, x: torch.Tensor, s: nv.ConvShape, *, dw: torch.Tensor,
                    accumulate: bool = True, policy: "nv.GemmPolicy | None" = None) -> torch.Tensor:
    OH, OW = conv_out_hw(s.H, s.W, s.KH, s.stride, s.pad)
    _conv_check_x(x, s, dy.dtype, "conv_bwd_weight")
    _check(dy.is_contiguous() and tuple(dy.shape) == (s.B, OH, OW, s.Cout), "conv_bwd_weight: dy shape")
    _check(dw.dtype == torch.float32 and dw.is_contiguous() and tuple(dw.shape) == (s.Cout, s.Cin, s.KH, s.KW),
           "conv_bwd_weight: dw must be f32 [Cout,Cin,k,k]")
    if _pointwise(s, dy.dtype):
        M = s.B * s.H * s.W
        linear_wgrad(dy.view(M, s.Cout), x.view(M, s.Cs), out=dw.view(s.Cout, s.Cs), accumulate=accumulate,
                     compute_bf16=True, policy=policy)
        return dw
    nwork = value("sv_conv_bwd_weight_work_floats", ctypes.byref(s))
    work = torch.empty(nwork, device=dy.device, dtype=torch.float32)
    call("sv_conv_bwd_weight", ptr(dy), ptr(x), ptr(work), ptr(dw), int(accumulate), dt(dy), ctypes.byref(s),
         nv.pol_ref(policy))
    return dw


def image_u8_hwc_to_nhwc(img_u8: torch.Tensor, Cs: int, dtype: torch.dtype, *, mean=IMAGENET_MEAN,
                         std=IMAGENET_STD) -> torch.Tensor:
    """Device form of the classification transform tail (row f1): collated uint8 crops [B,H,W,3]
    (reference construct_3channel, training/datasets/classification.py:40-68) -> ToTensor -> Normalize
    -> the ResNet stem operand NHWC [B,H,W,Cs] (channels >= 3 zero)."""
    _check(img_u8.dtype == torch.uint8 and img_u8.dim() == 4 and img_u8.shape[-1] == 3 and img_u8.is_contiguous(),
           "image_u8_hwc_to_nhwc: expects contiguous uint8 [B,H,W,3]")
    B, H, W, _ = img_u8.shape
    _check((B * H * W) % 4 == 0, "image_u8_hwc_to_nhwc: B*H*W must be a multiple of 4")
    out = torch.empty(B, H, W, Cs, device=img_u8.device, dtype=dtype)
    call("sv_image_u8_hwc_to_nhwc", ptr(img_u8), _host3(mean), _host3(std), ptr(out), dt(out), B, H, W, Cs)
    return out


def image_to_nhwc(img: torch.Tensor, Cs: int, dtype: torch.dtype) -> torch.Tensor:
    B, C, H, W = img.shape
    _check(img.dtype == torch.float32 and img.is_contiguous() and Cs >= C, "image_to_nhwc: need contiguous f32 NCHW")
    out = torch.empty(B, H, W, Cs, device=img.device, dtype=dtype)
    call("sv_image_to_nhwc", ptr(img), ptr(out), dt(out), B, C, H, W, Cs)
    return out


def _bn_c_ok(C: int) -> bool:
    return C >= 4 and C % 4 == 0 and (C // 4 <= 256 or (C // 4) % 256 == 0)


def bn_stats(y2d: torch.Tensor, *, eps: float = EPS_BN, momentum: float = 0.1, running_mean=None, running_var=None,
             num_batches_tracked=None):
    """Train-mode batch statistics of y [rows, C] -> (mean, rstd) f32; running stats (and the int64
    num_batches_tracked counter) updated in place on the device."""
    rows, C = y2d.shape
    _check(_bn_c_ok(C) and y2d.is_contiguous() and rows > 0, f"bn_stats: unsupported C={C}")
    P = value("sv_bn_nparts", rows, C)
    part = torch.empty(P, 2, C, device=y2d.device, dtype=torch.float32)
    call("sv_bn_stats", ptr(y2d), dt(y2d), rows, C, ptr(part))
    mean = torch.empty(C, device=y2d.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    _fin("sv_bn_stats_finish", ptr(y2d), dt(y2d), ptr(part), P, rows, C, float(eps), float(momentum), ptr(mean),
         ptr(rstd), ptr(running_mean), ptr(running_var), ptr(num_batches_tracked), *_fin_ws(part.device))
    return mean, rstd


def bn_eval_params(running_mean: torch.Tensor, running_var: torch.Tensor, eps: float = EPS_BN):
    C = running_mean.numel()
    mean = torch.empty(C, device=running_mean.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    call("sv_bn_eval_params", ptr(running_mean), ptr(running_var), float(eps), ptr(mean), ptr(rstd), C)
    return mean, rstd


def bn_act(y2d, mean, rstd, gamma, beta, *, res=None, res_bn=None, relu=True, out_dtype=torch.float32,
           out=None) -> torch.Tensor:
    """act(gamma (y-mean) rstd + beta + r), r = res or BN(res) with res_bn = (mean, rstd, gamma, beta)."""
    rows, C = y2d.shape
    _check(C % 4 == 0 and y2d.is_contiguous(), "bn_act: C must be a multiple of 4")
    if res is not None:
        _check(res.is_contiguous() and res.numel() == rows * C, "bn_act: residual shape")
    rm, rr, rg, rb = res_bn if res_bn is not None else (None, None, None, None)
    if out is None:
        out = torch.empty(rows, C, device=y2d.device, dtype=out_dtype)
    _fin("sv_bn_act_fwd", ptr(y2d), dt(y2d), ptr(mean), ptr(rstd), ptr(gamma), ptr(beta), ptr(res),
         nv.dt_none(res), ptr(rm), ptr(rr), ptr(rg), ptr(rb), int(relu), ptr(out), dt(out), rows, C)
    return out


# One launch per BatchNorm where the rows are few (sv_bn_*_small: ResNet layers 3-4 at 256 px), bit for bit the
# multi-launch path.  Opt-in (SV_BN_SMALL=1): measured slower (classification 3524-3542 vs 3779-3806 img/s
# interleaved, profiles/round4/r8c_bn_small_ab.txt).  A workgroup that owns 8 channels over all rows reads 16 B per
# row, one cache line per lane, so it streams at the L1's line rate: layer3's output BatchNorm backward took 86 us
# in one launch against ~45 us in three; at layer4 the two forms are equal (r8d trace)
_BN_SMALL = os.environ.get("SV_BN_SMALL", "0") != "0"
_SMALL_OK: dict = {}


def bn_small_ok(rows: int, C: int) -> bool:
    """Whether (rows, C) has the one-launch BatchNorm geometry (sv_bn_small_ok)."""
    key = (rows, C)
    ok = _SMALL_OK.get(key)
    if ok is None:
        ok = _SMALL_OK[key] = bool(value("sv_bn_small_ok", rows, C))
    return _BN_SMALL and ok


def _bn_small_args_ok(*ts) -> bool:
    return all(t is None or (t.is_cuda and t.is_contiguous() and t.data_ptr() % 16 == 0) for t in ts)


# The statistics fold inside the consuming pass (sv_bn_act_fold / sv_bn_bwd_apply_fold): one launch fewer per
# BatchNorm, bit for bit the separate fold.  Opt-in (SV_BN_FOLD=1): measured slower -- classification 2713-2718 vs
# 4076-4093 img/s with up to 2048 workgroups (their ticket / exit atomics on one counter serialise), and a graph-timed
# launch at 256 workgroups still 1.1-2.2x the separate finish + activation (profiles/round5/r11e_fold_bench.txt):
# the fold's round trips sit in front of every workgroup's first load.  The separate fold's chunks run in parallel
# workgroups instead (_fin_ws).
_BN_FOLD = os.environ.get("SV_BN_FOLD", "0") != "0"
_FOLD_OK: dict = {}
_FOLD_WS: dict = {}


def _fin_ws(device) -> tuple:
    """(ctl, ws) pointers for a separate fold launch on the current stream: its chunks of 1024 partials then fold in
    parallel workgroups (sv_bn_stats_finish / sv_bn_bwd_finish; same bits)."""
    ctl, ws = _fold_ws(device)
    return ptr(ctl), ptr(ws)


def bn_fold_ok(rows: int, C: int, nparts: int) -> bool:
    """Whether (rows, C, nparts) has the fold kernels' geometry (sv_bn_fold_ok), and SV_BN_FOLD is on."""
    key = (rows, C, nparts)
    ok = _FOLD_OK.get(key)
    if ok is None:
        ok = _FOLD_OK[key] = bool(value("sv_bn_fold_ok", rows, C, nparts))
    return _BN_FOLD and ok


def _fold_ws(device):
    """(ctl, ws) of the fold kernels on the current stream: the counters start zero and every launch leaves them
    zero; never reallocated (a captured graph keeps the pointers)."""
    key = (device, nv._stream())
    t = _FOLD_WS.get(key)
    if t is None:
        t = _FOLD_WS[key] = (torch.zeros(nv.SV_BN_FOLD_CTL_INTS, device=device, dtype=torch.int32),
                             torch.empty(nv.SV_BN_FOLD_WS_FLOATS, device=device, dtype=torch.float32))
    return t


def bn_fold_timeouts(device) -> int:
    """Fold-kernel polls that timed out on any stream of ``device`` since the workspaces were made (0 expected)."""
    return sum(int(ctl[3].item()) for (d, _), (ctl, _) in _FOLD_WS.items() if d == device)


def bn_act_fold(y2d, part, bn_params: tuple, *, res=None, res_part=None, res_params: tuple | None = None,
                relu=True, out_dtype=torch.float32):
    """bn_act_small's contract at any row count the fold kernels take (bn_fold_ok): the statistics fold of the conv
    epilogue's partials inside the activation pass (sv_bn_act_fold) -- bit for bit ``bn_stats_from_partials`` +
    ``bn_act``.  -> (out, mean, rstd[, mean2, rstd2])."""
    rows, C = y2d.shape
    g, b, eps, mom, rm, rv, nbt = bn_params
    dev = y2d.device
    mean = torch.empty(C, device=dev, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    out = torch.empty(rows, C, device=dev, dtype=out_dtype)
    if res_part is not None:
        g2, b2, eps2, mom2, rm2, rv2, nbt2 = res_params
        mean2, rstd2 = torch.empty_like(mean), torch.empty_like(mean)
    else:
        g2 = b2 = rm2 = rv2 = nbt2 = mean2 = rstd2 = None
        eps2, mom2 = 0.0, 0.0
    ctl, ws = _fold_ws(dev)
    _fin("sv_bn_act_fold", ptr(y2d), dt(y2d), ptr(part), part.shape[0], float(eps), float(mom), ptr(g), ptr(b),
         ptr(mean), ptr(rstd), ptr(rm), ptr(rv), ptr(nbt), ptr(res), nv.dt_none(res), ptr(res_part),
         res_part.shape[0] if res_part is not None else 0, float(eps2), float(mom2), ptr(g2), ptr(b2), ptr(mean2),
         ptr(rstd2), ptr(rm2), ptr(rv2), ptr(nbt2), int(relu), ptr(out), dt(out), rows, C, ptr(ctl), ptr(ws))
    if res_part is not None:
        return out, mean, rstd, mean2, rstd2
    return out, mean, rstd


def bn_act_partials(y2d, part, bn_params: tuple, *, res=None, res_part=None, res_params: tuple | None = None,
                    relu=True, out_dtype=torch.float32):
    """Train-mode BatchNorm (+ residual, + ReLU) from the conv epilogue's partials with the fewest launches the shape
    allows: bn_act_small (rows <= 8192, opt-in SV_BN_SMALL), bn_act_fold, else bn_stats_from_partials + bn_act.  All
    three give the same bits.  -> (out, mean, rstd[, mean2, rstd2])."""
    rows, C = y2d.shape
    args = (y2d, part, res, res_part) + bn_params[:2] + (res_params[:2] if res_params else ())
    if bn_small_ok(rows, C) and _bn_small_args_ok(*args):
        return bn_act_small(y2d, part, bn_params, res=res, res_part=res_part, res_params=res_params, relu=relu,
                            out_dtype=out_dtype)
    if (bn_fold_ok(rows, C, part.shape[0]) and _bn_small_args_ok(*args)
            and (res_part is None or res_part.shape[0] == part.shape[0])):
        return bn_act_fold(y2d, part, bn_params, res=res, res_part=res_part, res_params=res_params, relu=relu,
                           out_dtype=out_dtype)
    g, b, eps, mom, rm, rv, nbt = bn_params
    mean, rstd = bn_stats_from_partials(part, rows, eps=eps, momentum=mom, running_mean=rm, running_var=rv,
                                        num_batches_tracked=nbt)
    res_bn = None
    if res_part is not None:
        g2, b2, eps2, mom2, rm2, rv2, nbt2 = res_params
        mean2, rstd2 = bn_stats_from_partials(res_part, rows, eps=eps2, momentum=mom2, running_mean=rm2,
                                              running_var=rv2, num_batches_tracked=nbt2)
        res_bn = (mean2, rstd2, g2, b2)
    out = bn_act(y2d, mean, rstd, g, b, res=res, res_bn=res_bn, relu=relu, out_dtype=out_dtype)
    if res_part is not None:
        return out, mean, rstd, mean2, rstd2
    return out, mean, rstd


def bn_act_small(y2d, part, bn_params: tuple, *, res=None, res_part=None, res_params: tuple | None = None,
                 relu=True, out_dtype=torch.float32):
    """Train-mode BatchNorm (+ residual, + its own ReLU) from the conv epilogue's unshifted statistics partials in
    ONE launch (sv_bn_act_small): bit for bit ``bn_stats_from_partials`` + ``bn_act``.  ``bn_params`` =
    (gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked); with ``res_part`` the residual is
    the projection shortcut's conv output and ``res_params`` its BatchNorm's.  -> (out, mean, rstd[, mean2, rstd2])."""
    rows, C = y2d.shape
    g, b, eps, mom, rm, rv, nbt = bn_params
    dev = y2d.device
    mean = torch.empty(C, device=dev, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    out = torch.empty(rows, C, device=dev, dtype=out_dtype)
    if res_part is not None:
        g2, b2, eps2, mom2, rm2, rv2, nbt2 = res_params
        mean2, rstd2 = torch.empty_like(mean), torch.empty_like(mean)
    else:
        g2 = b2 = rm2 = rv2 = nbt2 = mean2 = rstd2 = None
        eps2, mom2 = 0.0, 0.0
    call("sv_bn_act_small", ptr(y2d), dt(y2d), ptr(part), part.shape[0], float(eps), float(mom), ptr(g), ptr(b),
         ptr(mean), ptr(rstd), ptr(rm), ptr(rv), ptr(nbt), ptr(res), nv.dt_none(res), ptr(res_part),
         res_part.shape[0] if res_part is not None else 0, float(eps2), float(mom2), ptr(g2), ptr(b2), ptr(mean2),
         ptr(rstd2), ptr(rm2), ptr(rv2), ptr(nbt2), int(relu), ptr(out), dt(out), rows, C)
    if res_part is not None:
        return out, mean, rstd, mean2, rstd2
    return out, mean, rstd


def bn_bwd(dout2d, y2d, mean, rstd, gamma, *, act=None, relu_beta=None, dgamma=None, dbeta=None,
           dx_dtype=torch.float32, gmask=None, mask_inplace: bool = False, batch_stats: bool = True,
           part: torch.Tensor | None = None) -> torch.Tensor:
    """BatchNorm backward with an optional ReLU mask on dout; dgamma/dbeta accumulate.  The mask is
    act > 0, or -- ``relu_beta`` = the BN's beta, for a BN followed by its own ReLU -- recomputed from y
    like the forward's pre-activation (sv_bn_relu_bwd_*: the activation is not read again).
    ``mask_inplace`` (act form, f32 or bf16 dout): the statistics pass overwrites dout with the masked gradient
    (sv_bn_bwd_stats_mask), which the apply pass then reads without the mask and the caller keeps as the
    shortcut's gradient; ``gmask`` instead writes it to a separate f32 buffer from the apply pass.
    ``batch_stats``: train mode (mean / rstd are the batch's own, so dx carries the two mean corrections);
    False: eval mode (running statistics, an affine map: dx = gamma * rstd * dout, the apply kernel reading
    zero correction sums).
    ``part`` (relu_beta form): the backward statistics' partials [P][2][C] already summed by the producer of
    dout (conv_bwd_data_bn), so the statistics pass is skipped."""
    rows, C = y2d.shape
    _check(_bn_c_ok(C) and dout2d.numel() == rows * C and dout2d.is_contiguous(), "bn_bwd: bad shapes")
    _check(act is None or relu_beta is None, "bn_bwd: act and relu_beta are exclusive")
    if act is not None:
        _check(act.numel() == rows * C and act.is_contiguous(), "bn_bwd: act shape")
    if gmask is not None:
        _check(gmask.dtype == torch.float32 and gmask.numel() == rows * C and relu_beta is None,
               "bn_bwd: gmask must be f32 [rows,C] (act-mask form only)")
    if mask_inplace:
        _check(act is not None and gmask is None and dout2d.dtype in (torch.float32, torch.bfloat16),
               "bn_bwd: mask_inplace needs act, an f32 / bf16 dout and no gmask")
    given = part is not None
    if given:
        _check(relu_beta is not None and part.dtype == torch.float32 and part.is_contiguous() and part.dim() == 3
               and tuple(part.shape[1:]) == (2, C), "bn_bwd: part must be f32 [P][2][C] (relu_beta form)")
    small_mode = (nv.SV_BN_SMALL_RELU if relu_beta is not None else nv.SV_BN_SMALL_MASK if mask_inplace else None)
    if (small_mode is not None and gmask is None and bn_small_ok(rows, C)
            and _bn_small_args_ok(dout2d, y2d, mean, rstd, gamma, act, relu_beta, part, dgamma, dbeta)):
        dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
        call("sv_bn_bwd_small", small_mode, ptr(dout2d), dt(dout2d), ptr(act), nv.dt_none(act), ptr(y2d), dt(y2d),
             ptr(mean), ptr(rstd), ptr(gamma), ptr(relu_beta), None, 0, None, None, None, ptr(part),
             part.shape[0] if given else 0, ptr(dx), None, dt(dx), ptr(dgamma), ptr(dbeta), None, None,
             int(batch_stats), rows, C)
        return dx
    if given:
        P = part.shape[0]
    else:
        P = value("sv_bn_nparts", rows, C)
        part = torch.empty(P, 2, C, device=y2d.device, dtype=torch.float32)
    if given:
        pass  # summed by dout's producer (conv_bwd_data_bn)
    elif relu_beta is not None:
        call("sv_bn_relu_bwd_stats", ptr(dout2d), dt(dout2d), ptr(y2d), dt(y2d), ptr(mean), ptr(rstd), ptr(gamma),
             ptr(relu_beta), rows, C, ptr(part))
    elif mask_inplace:
        call("sv_bn_bwd_stats_mask", ptr(dout2d), dt(dout2d), ptr(act), dt(act), ptr(y2d), dt(y2d), ptr(mean),
             ptr(rstd), rows, C, ptr(part))
        act = None  # dout now holds the masked gradient
    else:
        call("sv_bn_bwd_stats", ptr(dout2d), dt(dout2d), ptr(act), nv.dt_none(act), ptr(y2d), dt(y2d), ptr(mean),
             ptr(rstd), rows, C, ptr(part))
    if ((relu_beta is not None or act is None) and gmask is None and bn_fold_ok(rows, C, P)
            and _bn_small_args_ok(dout2d, y2d, mean, rstd, gamma, relu_beta, part)):
        # the finish inside the apply pass (sv_bn_bwd_apply_fold): MASK = dout already masked (mask_inplace)
        dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
        ctl, ws = _fold_ws(y2d.device)
        mode = nv.SV_BN_SMALL_RELU if relu_beta is not None else nv.SV_BN_SMALL_MASK
        _fin("sv_bn_bwd_apply_fold", mode, ptr(dout2d), dt(dout2d), None, 0, 0, ptr(y2d), dt(y2d), ptr(mean),
             ptr(rstd), ptr(gamma), ptr(relu_beta), None, 0, None, None, None, ptr(part), None, P, ptr(dx), None,
             dt(dx), ptr(dgamma), ptr(dbeta), None, None, int(batch_stats), rows, C, ptr(ctl), ptr(ws))
        return dx
    sums = torch.empty(2, C, device=y2d.device, dtype=torch.float32)
    _fin("sv_bn_bwd_finish", ptr(part), P, C, ptr(sums), ptr(dgamma), ptr(dbeta), *_fin_ws(part.device))
    if not batch_stats:
        sums.zero_()
    dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
    if relu_beta is not None:
        call("sv_bn_relu_bwd_apply", ptr(dout2d), dt(dout2d), ptr(y2d), dt(y2d), ptr(mean), ptr(rstd), ptr(gamma),
             ptr(relu_beta), ptr(sums), ptr(dx), dt(dx), rows, C)
    else:
        call("sv_bn_bwd_apply", ptr(dout2d), dt(dout2d), ptr(act), nv.dt_none(act), ptr(y2d), dt(y2d), ptr(mean),
             ptr(rstd), ptr(gamma), ptr(sums), ptr(dx), dt(dx), ptr(gmask), rows, C)
    return dx


def bn_bwd_dual(gm, y2d, mean, rstd, gamma, act, y2, mean2, rstd2, gamma2, *, dgamma=None, dbeta=None,
                dgamma2=None, dbeta2=None, dx_dtype=torch.float32, batch_stats: bool = True):
    """A projection-shortcut block's two output BatchNorms from one masked gradient: equals
    ``bn_bwd(gm, y2d, ..., act=act, mask_inplace=True)`` followed by ``bn_bwd(gm, y2, mean2, rstd2, gamma2)``
    bit for bit (gm, f32 or bf16, is overwritten with the masked gradient the same way), with gm read once per pass
    instead of twice (sv_bn_bwd_stats_mask_dual / sv_bn_bwd_apply_dual). -> (dx, dx2)."""
    rows, C = y2d.shape
    _check(_bn_c_ok(C) and gm.dtype in (torch.float32, torch.bfloat16) and gm.numel() == rows * C and gm.is_contiguous()
           and act.numel() == rows * C and act.is_contiguous() and y2.numel() == rows * C and y2.is_contiguous(),
           "bn_bwd_dual: bad shapes")
    if bn_small_ok(rows, C) and _bn_small_args_ok(gm, y2d, mean, rstd, gamma, act, y2, mean2, rstd2, gamma2, dgamma,
                                                   dbeta, dgamma2, dbeta2):
        dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
        dx2 = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
        call("sv_bn_bwd_small", nv.SV_BN_SMALL_DUAL, ptr(gm), dt(gm), ptr(act), dt(act), ptr(y2d), dt(y2d), ptr(mean),
             ptr(rstd), ptr(gamma), None, ptr(y2), dt(y2), ptr(mean2), ptr(rstd2), ptr(gamma2), None, 0, ptr(dx),
             ptr(dx2), dt(dx), ptr(dgamma), ptr(dbeta), ptr(dgamma2), ptr(dbeta2), int(batch_stats), rows, C)
        return dx, dx2
    P = value("sv_bn_nparts", rows, C)
    part = torch.empty(2, P, 2, C, device=y2d.device, dtype=torch.float32)
    call("sv_bn_bwd_stats_mask_dual", ptr(gm), dt(gm), ptr(act), dt(act), ptr(y2d), dt(y2d), ptr(mean), ptr(rstd),
         ptr(y2), dt(y2), ptr(mean2), ptr(rstd2), rows, C, ptr(part[0]), ptr(part[1]))
    if bn_fold_ok(rows, C, P) and _bn_small_args_ok(gm, y2d, mean, rstd, gamma, y2, mean2, rstd2, gamma2):
        dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
        dx2 = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
        ctl, ws = _fold_ws(y2d.device)
        _fin("sv_bn_bwd_apply_fold", nv.SV_BN_SMALL_DUAL, ptr(gm), dt(gm), None, 0, 0, ptr(y2d), dt(y2d), ptr(mean),
             ptr(rstd), ptr(gamma), None, ptr(y2), dt(y2), ptr(mean2), ptr(rstd2), ptr(gamma2), ptr(part[0]),
             ptr(part[1]), P, ptr(dx), ptr(dx2), dt(dx), ptr(dgamma), ptr(dbeta), ptr(dgamma2), ptr(dbeta2),
             int(batch_stats), rows, C, ptr(ctl), ptr(ws))
        return dx, dx2
    sums = torch.empty(2, 2, C, device=y2d.device, dtype=torch.float32)
    _fin("sv_bn_bwd_finish", ptr(part[0]), P, C, ptr(sums[0]), ptr(dgamma), ptr(dbeta), *_fin_ws(part.device))
    _fin("sv_bn_bwd_finish", ptr(part[1]), P, C, ptr(sums[1]), ptr(dgamma2), ptr(dbeta2), *_fin_ws(part.device))
    if not batch_stats:
        sums.zero_()
    dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
    dx2 = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
    call("sv_bn_bwd_apply_dual", ptr(gm), dt(gm), ptr(y2d), dt(y2d), ptr(mean), ptr(rstd), ptr(gamma), ptr(sums[0]),
         ptr(y2), dt(y2), ptr(mean2), ptr(rstd2), ptr(gamma2), ptr(sums[1]), ptr(dx), ptr(dx2), dt(dx), rows, C)
    return dx, dx2


def bn_relu_bwd_pooled(dpool4d: torch.Tensor, idx: torch.Tensor, H: int, W: int, y2d, mean, rstd, gamma, beta, *,
                       dgamma=None, dbeta=None, dx_dtype=torch.float32, batch_stats: bool = True) -> torch.Tensor:
    """bn_bwd(maxpool_bwd(dpool, idx, H, W), y, ..., relu_beta=beta) without materialising the max-pool
    backward: both BatchNorm passes gather it from dpool / idx (sv_bn_relu_bwd_*_pool), bit for bit."""
    B, OH, OW, C = dpool4d.shape
    rows = y2d.shape[0]
    _check(dpool4d.dtype in (torch.float32, torch.bfloat16) and dpool4d.is_contiguous() and idx.shape == dpool4d.shape
           and idx.is_contiguous() and (OH, OW) == conv_out_hw(H, W, 3, 2, 1) and rows == B * H * W
           and y2d.shape[1] == C and _bn_c_ok(C), "bn_relu_bwd_pooled: shape mismatch")
    P = value("sv_bn_nparts", rows, C)
    part = torch.empty(P, 2, C, device=y2d.device, dtype=torch.float32)
    call("sv_bn_relu_bwd_stats_pool", ptr(dpool4d), dt(dpool4d), ptr(idx), B, H, W, ptr(y2d), dt(y2d), ptr(mean),
         ptr(rstd), ptr(gamma), ptr(beta), C, ptr(part))
    if (bn_fold_ok(rows, C, P) and rows * C < 2 ** 31
            and _bn_small_args_ok(dpool4d, y2d, mean, rstd, gamma, beta)):
        dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
        ctl, ws = _fold_ws(y2d.device)
        _fin("sv_bn_bwd_apply_fold", nv.SV_BN_SMALL_RELU, ptr(dpool4d), dt(dpool4d), ptr(idx), H, W, ptr(y2d), dt(y2d),
             ptr(mean), ptr(rstd), ptr(gamma), ptr(beta), None, 0, None, None, None, ptr(part), None, P, ptr(dx),
             None, dt(dx), ptr(dgamma), ptr(dbeta), None, None, int(batch_stats), rows, C, ptr(ctl), ptr(ws))
        return dx
    sums = torch.empty(2, C, device=y2d.device, dtype=torch.float32)
    _fin("sv_bn_bwd_finish", ptr(part), P, C, ptr(sums), ptr(dgamma), ptr(dbeta), *_fin_ws(part.device))
    if not batch_stats:
        sums.zero_()
    dx = torch.empty(rows, C, device=y2d.device, dtype=dx_dtype)
    call("sv_bn_relu_bwd_apply_pool", ptr(dpool4d), dt(dpool4d), ptr(idx), B, H, W, ptr(y2d), dt(y2d), ptr(mean),
         ptr(rstd), ptr(gamma), ptr(beta), ptr(sums), ptr(dx), dt(dx), C)
    return dx


def head_loss(logits: torch.Tensor, specs: list) -> tuple:
    """The multi-task classification loss and its logits gradient in one launch (sv_head_loss).  ``specs``: one
    (kind, offset, ncls, weight, label_smoothing, target) per task, kind nv.SV_HEAD_CE (target int64 [B]) or
    nv.SV_HEAD_BCE (target f32 / bf16 [B][ncls]).  -> (loss 0-dim f32, dlogits [B][K] f32)."""
    _check(logits.dtype == torch.float32 and logits.dim() == 2 and logits.is_contiguous(), "head_loss: logits")
    B, Kc = logits.shape
    cover = 0
    tasks = []
    for kind, off, n, w, sm, t in specs:
        if kind == nv.SV_HEAD_CE:
            _check(t.dtype == torch.int64 and t.is_contiguous() and t.numel() == B, "head_loss: CE target int64 [B]")
        else:
            _check(t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous() and t.numel() == B * n,
                   "head_loss: BCE target f32 / bf16 [B][ncls]")
        tasks.append(nv.HeadTask(kind, off, n, float(w), float(sm), ptr(t), dt(t) if kind == nv.SV_HEAD_BCE else 0))
        cover += n
    loss = torch.empty((), device=logits.device, dtype=torch.float32)
    dl = (torch.empty_like if cover == Kc else torch.zeros_like)(logits)
    call("sv_head_loss", ptr(logits), B, Kc, (nv.HeadTask * len(tasks))(*tasks), len(tasks), ptr(loss), ptr(dl))
    return loss, dl


def maxpool_fwd(x4d: torch.Tensor):
    B, H, W, C = x4d.shape
    _check(x4d.is_contiguous() and C % 4 == 0, "maxpool_fwd: need contiguous NHWC, C % 4 == 0")
    OH, OW = conv_out_hw(H, W, 3, 2, 1)
    y = torch.empty(B, OH, OW, C, device=x4d.device, dtype=x4d.dtype)
    idx = torch.empty(B, OH, OW, C, device=x4d.device, dtype=torch.uint8)
    call("sv_maxpool3s2_fwd", ptr(x4d), dt(x4d), ptr(y), ptr(idx), B, H, W, C)
    return y, idx


def maxpool_bwd(dout4d: torch.Tensor, idx: torch.Tensor, H: int, W: int, dx_dtype=torch.float32) -> torch.Tensor:
    B, OH, OW, C = dout4d.shape
    _check(dout4d.is_contiguous() and idx.shape == dout4d.shape and (OH, OW) == conv_out_hw(H, W, 3, 2, 1),
           "maxpool_bwd: shape mismatch")
    dx = torch.empty(B, H, W, C, device=dout4d.device, dtype=dx_dtype)
    call("sv_maxpool3s2_bwd", ptr(dout4d), dt(dout4d), ptr(idx), ptr(dx), dt(dx), B, H, W, C)
    return dx


def avgpool_fwd(x4d: torch.Tensor) -> torch.Tensor:
    B, H, W, C = x4d.shape
    _check(x4d.is_contiguous() and C % 4 == 0, "avgpool_fwd: need contiguous NHWC, C % 4 == 0")
    feat = torch.empty(B, C, device=x4d.device, dtype=torch.float32)
    call("sv_avgpool_fwd", ptr(x4d), dt(x4d), ptr(feat), B, H * W, C)
    return feat


def avgpool_bwd(dfeat: torch.Tensor, shape: tuple, dx_dtype=torch.float32) -> torch.Tensor:
    B, H, W, C = shape
    dfeat = dfeat.float().contiguous()
    _check(tuple(dfeat.shape) == (B, C), "avgpool_bwd: dfeat shape")
    dx = torch.empty(B, H, W, C, device=dfeat.device, dtype=dx_dtype)
    call("sv_avgpool_bwd", ptr(dfeat), ptr(dx), dt(dx), B, H * W, C)
    return dx
