"""Fused MLP backward (sv_mlp_bwd) diagnostics: run-to-run determinism of the fused and the three-kernel path, and how
dz departs from the three-kernel path (elements differing, worst ratio to the dy-rounding-flip bound)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()

from test_mlp_fused_gpu import _bwd_fused, _bwd_ops, _bwd_unfused  # noqa: E402

if not torch.cuda.is_available():
    sys.exit("no GPU")
dev = torch.device("cuda:0")
for M in [int(a) for a in sys.argv[1:]] or [524288]:
    o = _bwd_ops(dev, M, 128, seed=M)
    f1, f2 = _bwd_fused(o), _bwd_fused(o)
    u1, u2 = _bwd_unfused(o), _bwd_unfused(o)
    torch.cuda.synchronize()
    print(f"M={M} fused deterministic: " + " ".join(str(torch.equal(a, b)) for a, b in zip(f1, f2)))
    print(f"M={M} unfused deterministic: " + " ".join(str(torch.equal(a, b)) for a, b in zip(u1, u2)))
    dz, rz, rdy = f1[1].float(), u1[1].float(), u1[4].float()
    dyu = rdy.abs() * 2.0**-7
    lw = o["lnw"][None, :]
    xh = ((o["z"].float() - o["mean"][:, None]) * o["rstd"][:, None]).abs()
    a0 = (lw * dyu).mean(1, keepdim=True)
    a1 = (lw * dyu * xh).mean(1, keepdim=True)
    tol = rz.abs() * 2.0**-7 + o["rstd"][:, None] * (lw * dyu + a0 + xh * a1)
    err = (dz - rz).abs()
    r = err / tol
    i = int(r.argmax())
    print(f"M={M} dz differing {float((dz != rz).float().mean()):.4f}, worst err/bound {float(r.max()):.3f} at row "
          f"{i // 128} col {i % 128} (err {float(err.view(-1)[i]):.3e} rz {float(rz.view(-1)[i]):.3e})")
