"""CPU: the torch.ops.ofx.* custom operators are registered with the declared mutations, propagate shapes
and dtypes under FakeTensorMode (no device, no kernel), and refuse CPU tensors (no CPU fallback)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from occlusionfusion_amd import ops


def test_all_ops_registered_with_mutations():
    sch = {n: str(getattr(torch.ops.ofx, n).default._schema) for n in ops.OPS}
    assert "Tensor(a0!) tsdf, Tensor(a1!) weight, Tensor(a2!)? color, Tensor(a3!)? n_updated" in sch["integrate"]
    for n in ("gn_solve", "gn_setup", "gn_linearize", "gn_step", "gn_finish"):
        assert sch[n].startswith(f"ofx::{n}(Tensor(a0!) state"), sch[n]
    assert "Tensor(a6!) A, Tensor(a7!) rhs" in sch["gn_linearize"]
    assert "!" not in sch["skin_points"] and "!" not in sch["deform_points"]


def test_fake_kernels():
    with FakeTensorMode():
        pts, nodes = torch.empty(1000, 3), torch.empty(37, 3)
        a, w, v = torch.ops.ofx.skin_points(pts, nodes, 0.05, 4)
        assert (a.shape, a.dtype, w.shape, w.dtype, v.shape, v.dtype) == \
            ((1000, 4), torch.int32, (1000, 4), torch.float32, (1000,), torch.bool)
        out = torch.ops.ofx.deform_points(pts, a, w, v, torch.empty(37, 16), False)
        assert out.shape == (1000, 3) and out.dtype == torch.float32
        st = torch.zeros(1, dtype=torch.int32)
        args = [nodes, torch.empty(37, 8, dtype=torch.int32), torch.empty(37, 8), nodes, torch.empty(37),
                pts, a, w, pts, None, None, None, None, [525.0, 525.0, 319.5, 223.5]]
        fp, ip = [0.0, 1.0, 0.5, 1.0, 1e-7, 1.0, 1e-6, 1e-5], [10, 0, 1000, 1, 0, 10]
        R, T, status, loss = torch.ops.ofx.gn_solve(st, 0, *args, fp, ip)
        assert (R.shape, T.shape, status.dtype, loss.shape, loss.dtype) == \
            ((37, 3, 3), (37, 3), torch.int32, (10, 4), torch.float64)
        info = torch.ops.ofx.gn_setup(st, 0, *args, fp, ip)
        assert info.shape == (2,) and info.dtype == torch.int64
        R2, _, _, loss2 = torch.ops.ofx.gn_finish(st, 0, 37, 10)
        assert R2.shape == (37, 3, 3) and loss2.shape == (10, 4)
        dd, nn, cc = torch.ops.ofx.raycast(torch.empty(512 * 8), torch.empty(512 * 8), None, [16, 16, 16],
                                           [0.0, 0.0, 1.0], 0.004, 0.04, [525.0, 525.0, 319.5, 223.5], 448, 640,
                                           0.1, 10.0)
        assert dd.shape == (448, 640) and nn.shape == (448, 640, 3) and cc.shape == (448, 640)
        vol = torch.empty(512 * 8)
        assert torch.ops.ofx.integrate(vol, vol.clone(), None, None, torch.empty(448, 640), None, [16, 16, 16],
                                       [0, 2], [0.0, 0.0, 1.0], 0.004, 0.04, 0, [525.0, 525.0, 319.5, 223.5], 1.0,
                                       None, 0, 1, None, 0, None, None, None, None, None) is None


def test_cpu_tensors_are_refused():
    with pytest.raises(NotImplementedError):
        torch.ops.ofx.skin_points(torch.zeros(3, 3), torch.zeros(5, 3), 0.05, 4)
    with pytest.raises(NotImplementedError):
        torch.ops.ofx.deform_points(torch.zeros(3, 3), torch.zeros(3, 4, dtype=torch.int32), torch.zeros(3, 4),
                                    None, torch.zeros(5, 16), False)
