"""Host-side class routing (CPU): which constructor arguments make FastGPLattice / FastGPDigitalNetB2 the
multitask class (multitask.py) and which stay on the single-task fused path.  The reference builds every
case with one class (abstract_gp.py:58-72); a single task with ONE all-zero derivative row and coefficient
1 has exactly the single-task kernel (rank-1 task factor 1, task noise 0: gram_matrix_tasks == 1), e.g.
the probnum25 paper's `derivatives=[torch.zeros((1, d))]` f-only fits."""
import torch

import fastgaussianprocesses_amd as F
from fastgaussianprocesses_amd.fast_gp import _trivial_derivatives, _wants_multitask


def test_trivial_derivatives():
    z = torch.zeros((1, 3), dtype=torch.int64)
    assert _trivial_derivatives(None, None)
    assert _trivial_derivatives([z], None)
    assert _trivial_derivatives(z, None)
    assert _trivial_derivatives(torch.zeros(3, dtype=torch.int64), None)
    assert _trivial_derivatives([z], [torch.ones(1)])
    assert not _trivial_derivatives([z], [2 * torch.ones(1)])
    assert not _trivial_derivatives([torch.zeros((2, 3), dtype=torch.int64)], None)   # K counted twice
    assert not _trivial_derivatives([torch.tensor([[1, 0, 0]])], None)
    assert not _trivial_derivatives([z, z], None)


def test_wants_multitask_routing():
    z = torch.zeros((1, 2), dtype=torch.int64)
    e = torch.tensor([[1, 0]])
    for cls in (F.FastGPLattice, F.FastGPDigitalNetB2):
        assert not _wants_multitask(cls, (2,), {})
        assert not _wants_multitask(cls, (2,), {"num_tasks": 1})
        assert not _wants_multitask(cls, (2,), {"num_tasks": 1, "derivatives": [z]})
        assert _wants_multitask(cls, (2,), {"num_tasks": 2})
        assert _wants_multitask(cls, (2,), {"num_tasks": 2, "derivatives": [z, e]})
        assert _wants_multitask(cls, (2,), {"num_tasks": 1, "derivatives": [e]})
        assert _wants_multitask(cls, (2,), {"derivatives_coeffs": [torch.tensor([0.5])]})
