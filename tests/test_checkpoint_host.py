"""Host logic of optimizer-state save / restore (zero_amd/checkpoint.py) and of the ZeRO-3 output
grad-tensor walk, on the CPU (no device): the header refuses another world size / rank /
variant / ownership, a plain torch state dict (no header) passes, torch's step encodings read
back, and the inner optimizer's loader is re-bound."""
import pytest
import torch

from zero_amd import checkpoint as ckpt


def test_header_roundtrip_and_mismatches():
    h = ckpt.header(2, 8, 3, [6, 7])
    ckpt.check_header({"zero_amd": dict(h)}, h)  # its own header passes
    ckpt.check_header({}, h)  # a plain torch state dict (no header) passes
    for k, v in (("world_size", 4), ("rank", 2), ("variant", 1), ("local_param_indices", [6])):
        with pytest.raises(ValueError, match=k):
            ckpt.check_header({"zero_amd": dict(h, **{k: v})}, h)
    with pytest.raises(ValueError, match="format"):
        ckpt.check_header({"zero_amd": dict(h, format=99)}, h)
    z3 = ckpt.header(3, 2, 0, [0], update=True)
    with pytest.raises(ValueError, match="update"):
        ckpt.check_header({"zero_amd": dict(z3, update=False)}, z3)


def test_step_encodings():
    assert ckpt.step_of({}) == 0
    assert ckpt.step_of({"step": 7}) == 7
    assert ckpt.step_of({"step": torch.tensor(12.0)}) == 12


def test_inner_loader_rebound_and_param_groups():
    p = torch.nn.Parameter(torch.zeros(3))
    opt = torch.optim.Adam([p], lr=1e-3)
    seen = []

    class Owner:
        optimizer = opt

        def load_state_dict(self, sd):
            seen.append(sd)

    ckpt.bind_inner_load(Owner())
    opt.load_state_dict({"marker": 1})
    assert seen == [{"marker": 1}]
    sd = torch.optim.Adam([p], lr=5e-4).state_dict()
    ckpt.load_param_groups(opt, sd)  # torch's own loader, hyper-parameters only
    assert opt.param_groups[0]["lr"] == 5e-4 and opt.param_groups[0]["params"] == [p]
    assert len(opt.state) == 0
    assert ckpt.inner_params(opt) == [p]


def test_zero3_grad_tensor_walk():
    from zero_amd.zero3 import _grad_tensors

    a = torch.ones(2, requires_grad=True) * 2
    b = torch.ones(2)
    c = torch.ones(1, requires_grad=True) + 1
    out = (a, [b, {"k": c}], None, 3)
    got = _grad_tensors(out)
    assert len(got) == 2 and any(t is a for t in got) and any(t is c for t in got)
    assert _grad_tensors(b) == []
