"""ctypes binding of ``libsv_kernels.so`` -- the C ABI declared in ``include/sv_kernels.h``.

The product path has no CPU or PyTorch fallback: if the library is missing, fails to load, or a
declared symbol is absent, every call raises.  Tensors cross the boundary as raw device pointers
(``tensor.data_ptr()``) and the work is enqueued on ``torch.cuda.current_stream()``.
"""

from __future__ import annotations

import ctypes
import os
import re
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SV_LIB_PATH") or os.path.join(_HERE, "libsv_kernels.so")  # override: A/B experiments
HEADER = os.path.join(os.path.dirname(_HERE), "include", "sv_kernels.h")

SV_F32, SV_BF16 = 0, 1
SV_IMG_F32_NCHW, SV_IMG_U8_GRAY = 0, 1
SV_BN_SMALL_MASK, SV_BN_SMALL_RELU, SV_BN_SMALL_DUAL = 0, 1, 2
SV_HEAD_CE, SV_HEAD_BCE = 0, 1
SV_BN_FOLD_CTL_INTS, SV_BN_FOLD_WS_FLOATS = 256, 2 * 2 * 2048 + 2 * 64 * 16 * 64  # include/sv_kernels.h
(SV_EPI_STORE, SV_EPI_BIAS_GELU2, SV_EPI_BIAS_GAMMA_RES, SV_EPI_GELU_GRAD, SV_EPI_SLAB, SV_EPI_BIAS_GELU_DUAL,
 SV_EPI_MUL_AUX, SV_EPI_BIAS_GELU, SV_EPI_STORE_STATS, SV_EPI_STORE_BN_BWD, SV_EPI_LN_BWD) = range(11)

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float


class BnRef(ctypes.Structure):
    """sv_bn_ref (include/sv_kernels.h): the BatchNorm of SV_EPI_STORE_BN_BWD / sv_gemm_slab_finish_bn_bwd."""
    _fields_ = [("mean", _p), ("rstd", _p), ("gamma", _p), ("beta", _p)]


class GemmPolicy(ctypes.Structure):
    """sv_gemm_policy (include/sv_kernels.h): the launch policy of ONE GEMM / convolution call (no process-wide
    GEMM state).  All zero = the measured per-shape dispatch on every CU."""
    _fields_ = [("impl", _i32), ("grid_cap", _i32), ("wg_per_cu", _i32), ("priority", _i32)]

    def __repr__(self) -> str:
        return (f"GemmPolicy(impl={self.impl}, grid_cap={self.grid_cap}, wg_per_cu={self.wg_per_cu}, "
                f"priority={self.priority})")


class CtxInfo(ctypes.Structure):
    """sv_ctx_info (include/sv_kernels.h): the per-device state the library sizes its launches by."""
    _fields_ = [("device", _i32), ("compute_units", _i32), ("lds_bytes_per_wg", _i32), ("xcds", _i32),
                ("lds_raised_kernels", _i32), ("refs", _i32), ("arch", ctypes.c_char * 32)]


def policy(impl: int = 0, grid_cap: int = 0, wg_per_cu: int = 0, priority: int = 0) -> GemmPolicy:
    return GemmPolicy(int(impl), int(grid_cap or 0), int(wg_per_cu), int(priority))


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", _i32), ("N", _i32), ("K", _i32),
        ("A", _p), ("a_dtype", _i32), ("a_kmajor", _i32), ("lda", _i64),
        ("B", _p), ("b_dtype", _i32), ("b_kmajor", _i32), ("ldb", _i64),
        ("a_scale_k", _p),
        ("epilogue", _i32),
        ("C", _p), ("c_dtype", _i32), ("ldc", _i64),
        ("C2", _p), ("c2_dtype", _i32),
        ("bias", _p),
        ("gamma", _p),
        ("aux", _p), ("aux_dtype", _i32), ("ld_aux", _i64),
        ("split_k", _i32),
        ("compute", _i32),
        ("bn", ctypes.POINTER(BnRef)),
        ("policy", GemmPolicy),
        ("fold_out", _p), ("fold_ld", _i64), ("fold_accumulate", _i32), ("fold_counters", _p),
    ]


class RedSeg(ctypes.Structure):
    """sv_red_seg (include/sv_kernels.h): one partial reduction of sv_reduce_partials_multi."""
    _fields_ = [("part", _p), ("out", _p), ("n", _i64), ("P", _i32), ("accumulate", _i32)]


class HeadTask(ctypes.Structure):
    """sv_head_task (include/sv_kernels.h): one task of sv_head_loss."""
    _fields_ = [("kind", _i32), ("offset", _i32), ("ncls", _i32), ("weight", _f32), ("label_smoothing", _f32),
                ("target", _p), ("target_dtype", _i32)]


SV_MAX_RED_SEGS = 8


class PackSeg(ctypes.Structure):
    """sv_pack_seg (include/sv_kernels.h): one weight pack of sv_conv_weight_pack_multi."""
    _fields_ = [("w", _p), ("wp", _p), ("Cout", _i32), ("Cin", _i32), ("T", _i32), ("Cs", _i32)]


SV_MAX_PACK_SEGS = 32


class ConvShape(ctypes.Structure):
    _fields_ = [("B", _i32), ("H", _i32), ("W", _i32), ("Cs", _i32), ("Cout", _i32), ("KH", _i32), ("KW", _i32),
                ("stride", _i32), ("pad", _i32), ("Cin", _i32)]


_CS = ctypes.POINTER(ConvShape)
_POL = ctypes.POINTER(GemmPolicy)

# name -> argtypes (restype is int for all entry points unless listed in _RESTYPES)
_SIGS = {
    "sv_version": [],
    "sv_ctx_create": [_i32, ctypes.POINTER(_p)],
    "sv_ctx_destroy": [_p],
    "sv_ctx_get_info": [_p, ctypes.POINTER(CtxInfo)],
    "sv_last_error_string": [],
    "sv_build_target": [],
    "sv_gemm": [ctypes.POINTER(GemmDesc), _p],
    "sv_stream_create_cu_reserved": [_i32, ctypes.POINTER(_i32), _i32, ctypes.POINTER(_p)],
    "sv_gemm_slab_finish": [_p, _i32, _i32, _i32, _p, _i32, _i64, _i32, _p, _p],
    "sv_gemm_slab_finish_bn_bwd": [_p, _i32, _i32, _i32, _p, _p, ctypes.POINTER(BnRef), _p, _p],
    "sv_mlp_fwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i32, _p],
    "sv_mlp_bwd_nparts": [_i64, _i32],
    "sv_mlp_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i32, _p],
    "sv_transpose_scale_bf16": [_p, _p, _p, _i32, _i32, _p],
    "sv_layernorm_fwd": [_p, _i32, _p, _p, _p, _i32, _p, _p, _i64, _i32, _f32, _p],
    "sv_layernorm_bwd_nparts": [_i64, _i32],
    "sv_layernorm_bwd": [_p, _i32, _p, _i32, _p, _p, _p, _p, _i32, _i32, _p, _p, _i64, _i32, _p],
    "sv_dwconv7_ln_fwd": [_p, _i32, _p, _p, _p, _p, _f32, _p, _i32, _p, _i32, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_dwconv7_bwd_data": [_p, _i32, _p, _p, _p, _i32, _i32, _i32, _i32, _i32, _p],
    "sv_dwconv7_fwd_mfma": [_p, _i32, _p, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_dwconv7_bwd_data_mfma": [_p, _p, _p, _p, _i32, _i32, _i32, _i32, _i32, _p],
    "sv_dwconv7_bwd_weight_mfma_nparts": [_i32, _i32, _i32, _i32],
    "sv_dwconv7_bwd_weight_mfma": [_p, _p, _i32, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_dwconv7_bwd_weight_nparts": [_i32, _i32, _i32, _i32],
    "sv_dwconv7_ln_fused_ok": [_i32, _i32, _i32, _i32, _i32, _i32, _i32],
    "sv_diag_group_sum": [_p, _p, _p, _i64, _i32, _p],
    "sv_dwconv7_bwd_weight": [_p, _i32, _p, _i32, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_stem_patchify_ln_fwd": [_p, _p, _p, _p, _p, _f32, _p, _i32, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_stem_patchify_ln_bwd_nparts": [_i32, _i32, _i32, _i32],
    "sv_stem_patchify_ln_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_stem_patchify": [_p, _i32, _p, _p, _p, _i32, _i32, _i32, _p],
    "sv_stem_weight_pack": [_p, _p, _i32, _p],
    "sv_normalize_u8_gray": [_p, _p, _p, _p, _i32, _i32, _i32, _p],
    "sv_augment_u8": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p],
    "sv_resize_u8": [_p, _p, _p, _i32, _i32, _i32, _i32, _p, _p],
    "sv_downsample_ln_patch2_fwd": [_p, _p, _p, _f32, _p, _i32, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_downsample_ln_patch2_bwd_nparts": [_i32, _i32, _i32, _i32],
    "sv_downsample_ln_patch2_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_pool_ln_fwd": [_p, _p, _p, _f32, _p, _p, _p, _p, _i32, _i32, _i32, _p],
    "sv_pool_ln_bwd": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _p],
    "sv_reduce_partials": [_p, _i32, _i32, _i64, _p, _f32, _i32, _p],
    "sv_reduce_partials_bf16": [_p, _i32, _i64, _p, _f32, _i32, _p],
    "sv_reduce_partials_pair": [_p, _i64, _p, _p, _i64, _p, _i32, _f32, _i32, _p],
    "sv_reduce_partials_multi": [ctypes.POINTER(RedSeg), _i32, _f32, _p],
    "sv_colsum_nparts": [_i64, _i32],
    "sv_colsum": [_p, _i32, _i64, _i32, _p, _p],
    "sv_layerscale_wgrad_finish": [_p, _p, _p, _p, _p, _p, _p, _p, _i32, _i32, _p],
    "sv_layerscale_wgrad_reduce_ws": [_i32, _i32],
    "sv_layerscale_wgrad_reduce": [_p, _p, _i32, _p, _p, _p, _p, _p, _p, _p, _i32, _i32, _p],
    "sv_layerscale_wgrad_reduce_bf16": [_p, _p, _i32, _p, _p, _p, _p, _p, _p, _i32, _i32, _p],
    "sv_layerscale_wgrad_fold_finish": [_p, _p, _i32, _p, _p, _p, _p, _p, _p, _i32, _i32, _p],
    "sv_sqnorm_nparts": [_i64],
    "sv_sqnorm_partial": [_p, _i64, _p, _p],
    "sv_clip_coef": [_p, _i32, _f32, _p, _p],
    "sv_adamw_flat": [_p, _p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32, _i32, _p, _p],
    "sv_adamw_flat_dev": [_p, _p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _p, _p, _p],
    "sv_scale_rows_bf16": [_p, _p, _p, _i32, _i32, _p],
    "sv_cast_f32_bf16": [_p, _p, _i64, _p],
    # ResNet
    "sv_conv_weight_pack": [_p, _p, _i32, _CS, _p],
    "sv_conv_weight_pack_multi": [ctypes.POINTER(PackSeg), _i32, _i32, _p],
    "sv_conv_fwd": [_p, _p, _p, _i32, _i32, _CS, _POL, _p],
    "sv_conv_fwd_stats": [_p, _p, _p, _i32, _i32, _CS, _p, _POL, _p],
    "sv_conv_bwd_data": [_p, _p, _p, _i32, _i32, _i32, _CS, _POL, _p],
    "sv_conv_fwd_split": [_p, _p, _p, _i32, _i32, _CS, _p, _p, _i32, _POL, _p],
    "sv_conv_bwd_data_split": [_p, _p, _p, _i32, _i32, _i32, _CS, _p, _i32, _POL, _p],
    "sv_conv_bwd_data_bn": [_p, _p, _p, _i32, _CS, _p, ctypes.POINTER(BnRef), _p, _p, _i32, _POL, _p],
    "sv_conv_bwd_weight_work_floats": [_CS],
    "sv_conv_bwd_weight": [_p, _p, _p, _p, _i32, _i32, _CS, _POL, _p],
    "sv_image_to_nhwc": [_p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _p],
    "sv_image_u8_hwc_to_nhwc": [_p, _p, _p, _p, _i32, _i32, _i32, _i32, _i32, _p],
    "sv_bn_nparts": [_i64, _i32],
    "sv_bn_stats": [_p, _i32, _i64, _i32, _p, _p],
    "sv_bn_stats_finish": [_p, _i32, _p, _i32, _i64, _i32, _f32, _f32, _p, _p, _p, _p, _p, _p, _p, _p],
    "sv_bn_eval_params": [_p, _p, _f32, _p, _p, _i32, _p],
    "sv_bn_act_fwd": [_p, _i32, _p, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _i32, _p, _i32, _i64, _i32, _p],
    "sv_bn_bwd_stats": [_p, _i32, _p, _i32, _p, _i32, _p, _p, _i64, _i32, _p, _p],
    "sv_bn_bwd_stats_mask": [_p, _i32, _p, _i32, _p, _i32, _p, _p, _i64, _i32, _p, _p],
    "sv_bn_bwd_finish": [_p, _i32, _i32, _p, _p, _p, _p, _p, _p],
    "sv_bn_bwd_stats_mask_dual": [_p, _i32, _p, _i32, _p, _i32, _p, _p, _p, _i32, _p, _p, _i64, _i32, _p, _p, _p],
    "sv_bn_bwd_apply_dual": [_p, _i32, _p, _i32, _p, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _p, _p, _i32, _i64, _i32,
                             _p],
    "sv_bn_relu_bwd_stats": [_p, _i32, _p, _i32, _p, _p, _p, _p, _i64, _i32, _p, _p],
    "sv_bn_relu_bwd_apply": [_p, _i32, _p, _i32, _p, _p, _p, _p, _p, _p, _i32, _i64, _i32, _p],
    "sv_bn_relu_bwd_stats_pool": [_p, _i32, _p, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _p, _i32, _p, _p],
    "sv_bn_relu_bwd_apply_pool": [_p, _i32, _p, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _p, _p, _p, _i32, _i32, _p],
    "sv_bn_bwd_apply": [_p, _i32, _p, _i32, _p, _i32, _p, _p, _p, _p, _p, _i32, _p, _i64, _i32, _p],
    "sv_bn_small_ok": [_i64, _i32],
    "sv_bn_bwd_small": [_i32, _p, _i32, _p, _i32, _p, _i32, _p, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _i32, _p, _p,
                        _i32, _p, _p, _p, _p, _i32, _i64, _i32, _p],
    "sv_bn_act_small": [_p, _i32, _p, _i32, _f32, _f32, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _p, _i32, _f32, _f32,
                        _p, _p, _p, _p, _p, _p, _p, _i32, _p, _i32, _i64, _i32, _p],
    "sv_bn_fold_ok": [_i64, _i32, _i32],
    "sv_bn_act_fold": [_p, _i32, _p, _i32, _f32, _f32, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _p, _i32, _f32, _f32,
                       _p, _p, _p, _p, _p, _p, _p, _i32, _p, _i32, _i64, _i32, _p, _p, _p],
    "sv_bn_bwd_apply_fold": [_i32, _p, _i32, _p, _i32, _i32, _p, _i32, _p, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _p,
                             _i32, _p, _p, _i32, _p, _p, _p, _p, _i32, _i64, _i32, _p, _p, _p],
    "sv_head_loss": [_p, _i32, _i32, _p, _i32, _p, _p, _p],
    "sv_relu_mask": [_p, _i32, _p, _i32, _p, _i64, _p],
    "sv_maxpool3s2_fwd": [_p, _i32, _p, _p, _i32, _i32, _i32, _i32, _p],
    "sv_maxpool3s2_bwd": [_p, _i32, _p, _p, _i32, _i32, _i32, _i32, _i32, _p],
    "sv_avgpool_fwd": [_p, _i32, _p, _i32, _i32, _i32, _p],
    "sv_avgpool_bwd": [_p, _p, _i32, _i32, _i32, _i32, _p],
}
_RESTYPES = {"sv_last_error_string": ctypes.c_char_p, "sv_build_target": ctypes.c_char_p,
             "sv_conv_bwd_weight_work_floats": ctypes.c_int64}
# entry points that return a value (size / count) rather than an sv_status
_VALUE_FNS = {n for n in _SIGS if n.endswith(("_nparts", "_ws"))} | {"sv_version", "sv_bn_fold_ok", "sv_dwconv7_ln_fused_ok", "sv_conv_bwd_weight_work_floats",
                                                                     "sv_stream_create_cu_reserved", "sv_bn_small_ok"}

# entry points that take no stream (call() appends none) but return an sv_status
_NOSTREAM_FNS = {"sv_ctx_create", "sv_ctx_destroy", "sv_ctx_get_info"}

_lib = None
_lock = threading.Lock()


def header_symbols(path: str = HEADER) -> list[str]:
    """Every ``sv_*`` function declared in include/sv_kernels.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sv_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Load the kernel library (once) and bind every declared entry point.  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"spine_vision_amd: native kernel library not found at {LIB_PATH}; "
                "run `python __graft_entry__.py` (hipcc --offload-arch=gfx950) first"
            )
        L = ctypes.CDLL(LIB_PATH)
        missing = [s for s in header_symbols() if not hasattr(L, s)]
        if missing:
            raise RuntimeError(f"spine_vision_amd: {LIB_PATH} lacks symbols {missing}")
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
        return L


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_device = torch._C._cuda_getDevice


def _stream() -> int:
    """hipStream_t of the current stream of the current device (torch.cuda.current_stream().cuda_stream
    without its Python-level device lookup: ~6 us of host time per launch saved)."""
    return _raw_stream(_cur_device())


# ---- intra-device stream hand-offs without the system-scope fence -------------------------------------------------
# torch's stream events are hipEventDisableTiming events: recording one performs a SYSTEM-scope release (L2 writeback
# and invalidate, for host visibility) between the two kernels around it.  A hand-off between two streams of one
# device needs no host visibility: the producing kernel's own end-of-dispatch release already makes its writes visible
# device-wide.  These events add hipEventDisableSystemFence (hip_runtime_api.h), from a ring (a stream's wait binds
# to the record current at the hipStreamWaitEvent call, so a later re-record does not affect it).  Measured neutral on
# the ConvNeXt step (r13p, interleaved: 1142.0 / 1146.6 fenceless vs 1146.7 / 1144.6 img/s; the ~17 us main-queue gap
# before each block's depthwise backward-data stayed), so torch's events stay the default; SV_FENCELESS_EVENTS=1 (A/B).
FENCELESS_EVENTS = os.environ.get("SV_FENCELESS_EVENTS", "0") != "0"
_HIP_EVENT_DISABLE_TIMING, _HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x2, 0x20000000
_HIPRT = None
_RING: dict = {}


def _hiprt():
    """The HIP runtime torch loaded (one per process: bind to that library, not another copy)."""
    global _HIPRT
    if _HIPRT is None:
        path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
        h = ctypes.CDLL(path)
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        h.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        _HIPRT = h
    return _HIPRT


def handoff(src: torch.cuda.Stream, dst: torch.cuda.Stream) -> None:
    """dst waits for everything enqueued on src so far (src and dst on one device)."""
    if not FENCELESS_EVENTS:
        dst.wait_event(src.record_event())
        return
    h = _hiprt()
    key = src.device
    ring = _RING.get(key)
    if ring is None:
        ring = _RING[key] = [[], 0]
        with torch.cuda.device(src.device):
            for _ in range(256):
                ev = ctypes.c_void_p()
                rc = h.hipEventCreateWithFlags(ctypes.byref(ev), _HIP_EVENT_DISABLE_TIMING | _HIP_EVENT_DISABLE_SYSTEM_FENCE)
                if rc != 0:
                    raise RuntimeError(f"hipEventCreateWithFlags failed ({rc})")
                ring[0].append(ev)
    ev = ring[0][ring[1]]
    ring[1] = (ring[1] + 1) % len(ring[0])
    rc = h.hipEventRecord(ev, ctypes.c_void_p(src.cuda_stream))
    if rc == 0:
        rc = h.hipStreamWaitEvent(ctypes.c_void_p(dst.cuda_stream), ev, 0)
    if rc != 0:
        raise RuntimeError(f"stream hand-off failed (hip error {rc})")


_FNS: dict = {}  # name -> bound ctypes function (ctypes attribute lookup is a dict miss + a getattr per call)


class StreamProbe:
    """HIP events around every sv_* launch enqueued on one stream (bench.py: the main queue's busy time per step --
    the critical path of the two-stream backward -- measured live; torch's own kernels on that stream are not
    bracketed)."""

    def __init__(self, stream: torch.cuda.Stream) -> None:
        self.handle = stream.cuda_stream
        self.events: list = []

    def busy_ms(self) -> float:
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.events)

    def span_ms(self) -> float:
        torch.cuda.synchronize()
        return self.events[0][0].elapsed_time(self.events[-1][1]) if self.events else 0.0


STREAM_PROBE: StreamProbe | None = None


def call(name: str, *args):
    """Invoke an sv_* entry point on the current stream; raise RuntimeError on a non-zero status."""
    fn = _FNS.get(name)
    if fn is None:
        fn = _FNS[name] = getattr(_lib if _lib is not None else lib(), name)
    if name in _VALUE_FNS:
        return fn(*args)
    if name in _NOSTREAM_FNS:
        rc = fn(*args)
    else:
        s = _stream()
        pr = STREAM_PROBE
        if pr is not None and s == pr.handle:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(*args, s)
            e1.record()
            pr.events.append((e0, e1))
        else:
            rc = fn(*args, s)
    if rc != 0:
        msg = lib().sv_last_error_string().decode()
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")
    return rc


def value(name: str, *args) -> int:
    return getattr(lib(), name)(*args)


def pol_ref(p: GemmPolicy | None):
    """ctypes argument for a nullable ``const sv_gemm_policy*`` (None -> NULL = the defaults)."""
    return None if p is None else ctypes.byref(p)


def ptr(t: torch.Tensor | None) -> int | None:
    """Device pointer of a tensor (None -> NULL); refuses CPU tensors loudly."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("spine_vision_amd kernels need device tensors (got a CPU tensor)")
    return t.data_ptr()


def dt_none(t: torch.Tensor | None) -> int:
    return SV_F32 if t is None else dt(t)


def dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return SV_F32
    if t.dtype == torch.bfloat16:
        return SV_BF16
    raise TypeError(f"unsupported dtype {t.dtype}")


class DeviceContext:
    """The library's per-device context (sv_ctx): created once per device by the host (StepEngine,
    the trainers), it queries the device's properties up front and holds a reference until ``close()``.  Entry
    points find their device from the stream, so launches work with or without one."""

    def __init__(self, device: int) -> None:
        h = _p()
        call("sv_ctx_create", int(device), ctypes.byref(h))
        self._h = h

    def info(self) -> CtxInfo:
        out = CtxInfo()
        call("sv_ctx_get_info", self._h, ctypes.byref(out))
        return out

    @property
    def handle(self) -> int:
        return int(self._h.value or 0)

    def close(self) -> None:
        if self._h is not None:
            call("sv_ctx_destroy", self._h)
            self._h = None


_CONTEXTS: dict = {}


def device_context(device: int) -> DeviceContext:
    """The process's context of ``device`` (created on first use, kept for the process's lifetime)."""
    c = _CONTEXTS.get(device)
    if c is None:
        c = _CONTEXTS[device] = DeviceContext(device)
    return c
