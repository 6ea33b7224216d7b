"""training.engine.ParamGate on CPU: the optimizer chunks follow the backbone's parameter groups in arena order (one
chunk per group, the model's heads in the last), a module maps to the chunk that holds its last parameter, groups out of
arena order are refused, and with no update in flight the waits are no-ops."""
import pytest
import torch.nn as nn

from spine_vision_amd.training.engine import ParamGate
from spine_vision_amd.training.flat import FlatArena, _align


class _Backbone(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Linear(3, 5)
        self.stages = nn.Sequential(nn.Linear(5, 7), nn.Identity(), nn.Linear(7, 9))
        self.head = nn.LayerNorm(9)

    def param_gate_groups(self):
        return [self.stem, *self.stages, self.head]


class _Model(nn.Module):
    def __init__(self):
        super().__init__()
        self.backbone = _Backbone()
        self.heads = nn.Linear(9, 2)


def test_chunks_follow_the_groups():
    m = _Model()
    a = FlatArena(m, "cpu", with_shadow=False)
    g = ParamGate(a, m.backbone.param_gate_groups())
    ends = []
    off = 0
    for mod in (m.backbone.stem, m.backbone.stages[0], m.backbone.stages[2], m.backbone.head):
        for p in mod.parameters():
            off += _align(p.numel())
        ends.append(off - _align(list(mod.parameters())[-1].numel()) + list(mod.parameters())[-1].numel())
    assert g.bounds == ends + [a.numel]  # the Identity stage holds nothing: no chunk
    assert g._chunk[id(m.backbone.stem)] == 0 and g._chunk[id(m.backbone.stages[2])] == 2
    assert g._chunk[id(m.backbone.head)] == 3 and id(m.backbone.stages[1]) not in g._chunk
    g.wait(m.backbone.stem)  # nothing in flight: no-op (no CUDA needed)
    g.wait_all()


def test_groups_out_of_arena_order_are_refused():
    m = _Model()
    a = FlatArena(m, "cpu", with_shadow=False)
    bb = m.backbone
    with pytest.raises(ValueError):
        ParamGate(a, [bb.stages[2], bb.stem])
