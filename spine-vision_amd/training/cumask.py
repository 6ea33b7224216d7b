"""CU-reserved compute streams for data-parallel runs (DESIGN.md "Multi-GPU").

A persistent v9 GEMM workgroup holds a whole CU (128-160 KiB of LDS) for its entire launch, and the lean
backward runs GEMMs on two streams at once, so a per-launch grid cap alone cannot keep CUs free for RCCL: two
capped grids together still cover the chip (tools/cu_mask_probe.py).  Under data parallelism the training step
therefore runs on streams created with a hardware CU mask (``sv_stream_create_cu_reserved``, over
hipExtStreamCreateWithCUMask) that excludes ``reserve`` CUs: no compute kernel of the step -- GEMM, depthwise,
LayerNorm, fold -- can occupy them, and RCCL's kernels, on their own unmasked streams, always find a CU.
"""

from __future__ import annotations

import ctypes

import torch

from .. import native as nv


def reserve_bits(ncu: int, reserve: int, pattern: str = "tail") -> list[int]:
    """CU indices to keep free: ``tail`` = the last ``reserve`` bits of the mask; ``strided`` = every
    (ncu / reserve)-th bit.  The runtime deals consecutive mask bits over the XCDs, so ``tail`` frees reserve / 8
    CUs on every XCD, while ``strided`` (stride 8) would mask out one whole XCD: the workgroups dealt to it then
    wait, measured 4x the comm latency and -12% step (tools/cu_mask_probe.py, profiles/round4/r7b_*, r7c_*)."""
    if reserve <= 0:
        return []
    if pattern == "tail":
        return list(range(ncu - reserve, ncu))
    step = max(1, ncu // reserve)
    return [i * step + step - 1 for i in range(reserve)]


_STREAMS: dict = {}


def masked_stream(device, reserved: list[int]) -> torch.cuda.ExternalStream:
    """A new torch stream on ``device`` whose kernels never run on the ``reserved`` CUs (lives until exit)."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    arr = (ctypes.c_int32 * max(1, len(reserved)))(*reserved)
    out = ctypes.c_void_p()
    rc = nv.value("sv_stream_create_cu_reserved", idx, arr, len(reserved), ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(f"sv_stream_create_cu_reserved failed: {nv.lib().sv_last_error_string().decode()}")
    return torch.cuda.ExternalStream(out.value, device=device)


def reserved_stream(device, reserve: int, role: str = "main", pattern: str = "tail") -> torch.cuda.ExternalStream:
    """The process's CU-reserved stream for ``role`` ("main" / "side") on ``device`` (created once)."""
    device = torch.device(device)
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    key = (device, role, reserve, pattern)
    if key not in _STREAMS:
        _STREAMS[key] = masked_stream(device, reserve_bits(ncu, reserve, pattern))
    return _STREAMS[key]
