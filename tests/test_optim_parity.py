"""Fused arena optimizers pinned against ``torch.optim`` over several steps, with weight
decay, momentum and nesterov -- on the CPU path and (``gpu``) on the HIP kernels.

Keras-semantics parity (TF's own optimizers) is unpinned: TensorFlow is not importable
here.  The update rules are written to coincide with torch.optim's for the options
used below (coupled L2 for SGD/Adam/RMSprop, decoupled for AdamW, eps outside the
square root)."""
import pytest
import torch

from cloud_amd import optim

CASES = {
    "sgd": (lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-2),
            lambda m: optim.SGD(m, learning_rate=0.1, momentum=0.9, weight_decay=1e-2)),
    "sgd_plain": (lambda ps: torch.optim.SGD(ps, lr=0.05),
                  lambda m: optim.SGD(m, learning_rate=0.05)),
    "sgd_nesterov": (lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-3),
                     lambda m: optim.SGD(m, learning_rate=0.1, momentum=0.9, nesterov=True, weight_decay=1e-3)),
    "adam": (lambda ps: torch.optim.Adam(ps, lr=1e-2, eps=1e-7, weight_decay=1e-3),
             lambda m: optim.Adam(m, learning_rate=1e-2, weight_decay=1e-3)),
    "adamw": (lambda ps: torch.optim.AdamW(ps, lr=1e-2, eps=1e-7, weight_decay=1e-2),
              lambda m: optim.AdamW(m, learning_rate=1e-2, weight_decay=1e-2)),
    "rmsprop": (lambda ps: torch.optim.RMSprop(ps, lr=1e-2, alpha=0.9, eps=1e-7, momentum=0.5, weight_decay=1e-3),
                lambda m: optim.RMSprop(m, learning_rate=1e-2, momentum=0.5, weight_decay=1e-3)),
}


def _run(kind, device, bf16_layer):
    torch.manual_seed(11)
    ours = torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.Linear(65, 7)).to(device)
    ref = torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.Linear(65, 7)).to(device)
    ref.load_state_dict(ours.state_dict())
    if bf16_layer:  # bf16 model copy + fp32 master (the framework's mixed-precision layout)
        ours[0].weight.data = ours[0].weight.data.to(torch.bfloat16)
        ref[0].weight.data = ours[0].weight.data.float()
    mk_ref, mk_ours = CASES[kind]
    o_ours = mk_ours(ours)
    # the arenas decay matrices only (biases / 1-D params sit in the non-decayed segment)
    o_ref = mk_ref([{"params": [p for p in ref.parameters() if p.ndim > 1]},
                    {"params": [p for p in ref.parameters() if p.ndim <= 1], "weight_decay": 0.0}])
    gen = torch.Generator().manual_seed(5)
    for step in range(5):
        o_ref.zero_grad()
        o_ours.zero_grad()
        for p_o, p_r in zip(ours.parameters(), ref.parameters()):
            g = torch.randn(p_r.shape, generator=gen).to(device)
            p_o.grad.copy_(g.to(p_o.grad.dtype))
            p_r.grad = p_o.grad.detach().float().clone()  # the same (possibly bf16-rounded) gradient
        o_ours.step()
        o_ref.step()
    for a in o_ours.arenas:
        for s in a.slots:
            want = dict(zip([id(p) for p in ours.parameters()], ref.parameters()))[id(s.param)]
            got = a.master[s.offset:s.offset + s.numel].reshape(want.shape)
            torch.testing.assert_close(got, want.detach(), atol=2e-6, rtol=2e-5)


@pytest.mark.parametrize("bf16_layer", [False, True])
@pytest.mark.parametrize("kind", sorted(CASES))
def test_cpu_path_matches_torch_optim(kind, bf16_layer):
    _run(kind, "cpu", bf16_layer)


@pytest.mark.gpu
@pytest.mark.parametrize("bf16_layer", [False, True])
@pytest.mark.parametrize("kind", sorted(CASES))
def test_hip_kernels_match_torch_optim(kind, bf16_layer):
    from cloud_amd.ops import _ext

    _ext.load(required=True)
    _run(kind, "cuda", bf16_layer)
