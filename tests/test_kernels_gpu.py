"""Numerics of the gfx950 HIP kernels vs plain PyTorch fp32 references.

Each test runs the HIP path (CUDA tensors, CLOUD_AMD_OPS=native) and compares
against the same op computed in fp32 with stock PyTorch on the same inputs.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ext_loaded():
    from cloud_amd.ops import _ext

    assert _ext.load(required=True) is not None


def test_extension_loads():
    _ext_loaded()
    import cloud_amd._C as C

    assert C.ARCH == "gfx950"


@pytest.mark.parametrize("shape", [(8, 14, 14, 64), (4, 7, 7, 2048), (2, 56, 56, 256), (3, 5, 5, 24)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_act_fwd_bwd(shape, relu, res):
    from cloud_amd.ops import bn_act

    torch.manual_seed(0)
    C = shape[-1]
    x = (torch.randn(shape, device=DEV) * 2 + 0.5).to(torch.bfloat16).requires_grad_()
    r = torch.randn(shape, device=DEV).to(torch.bfloat16).requires_grad_() if res else None
    g = (torch.rand(C, device=DEV) + 0.5).requires_grad_()
    b = torch.randn(C, device=DEV).requires_grad_()
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    y = bn_act(x, g, b, rm, rv, residual=r, relu=relu)
    dy = torch.randn(shape, device=DEV).to(torch.bfloat16)
    y.backward(dy)

    # fp32 reference
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    gr, br = g.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yr = F.batch_norm(xr.reshape(-1, C), rm2, rv2, gr, br, training=True, momentum=0.1, eps=1e-5).reshape(shape)
    if res:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=5e-2)
    torch.testing.assert_close(g.grad, gr.grad, atol=5e-2 * (x.numel() / C) ** 0.5, rtol=2e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=5e-2 * (x.numel() / C) ** 0.5, rtol=2e-2)
    if res:
        torch.testing.assert_close(r.grad.float(), rr.grad, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(rm, rm2, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(rv, rv2, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("B,C", [(256, 1000), (64, 10), (7, 130)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_softmax_xent(B, C, dtype):
    from cloud_amd.ops import softmax_cross_entropy

    torch.manual_seed(1)
    z = (torch.randn(B, C, device=DEV) * 3).to(dtype).requires_grad_()
    y = torch.randint(0, C, (B,), device=DEV)
    loss, correct = softmax_cross_entropy(z, y, denom=B)
    loss.backward()
    zr = z.detach().float().requires_grad_()
    lr = F.cross_entropy(zr, y)
    lr.backward()
    torch.testing.assert_close(loss.float(), lr, atol=1e-3, rtol=1e-3)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(z.grad.float(), zr.grad, atol=tol / B, rtol=tol)
    assert torch.equal(correct.bool(), zr.argmax(-1) == y)


def test_maxpool_and_gap():
    from cloud_amd.ops import global_avg_pool_nhwc, max_pool2d_nhwc

    torch.manual_seed(2)
    x = torch.randn(4, 17, 18, 64, device=DEV).to(torch.bfloat16).requires_grad_()
    y = max_pool2d_nhwc(x, 3, 2, 1)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    yr = F.max_pool2d(xr, 3, 2, 1)
    torch.testing.assert_close(y.float(), yr.permute(0, 2, 3, 1), atol=0, rtol=0)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=2e-2, rtol=2e-2)
    # generic gather path (not the 3x3/2/1 specialisation)
    x3 = torch.randn(2, 9, 10, 16, device=DEV).to(torch.bfloat16).requires_grad_()
    y3 = max_pool2d_nhwc(x3, 2, 2, 0)
    x3r = x3.detach().float().permute(0, 3, 1, 2).requires_grad_()
    y3r = F.max_pool2d(x3r, 2, 2, 0)
    dy3 = torch.randn_like(y3)
    y3.backward(dy3)
    y3r.backward(dy3.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(x3.grad.float(), x3r.grad.permute(0, 2, 3, 1), atol=2e-2, rtol=2e-2)

    x2 = torch.randn(5, 7, 7, 256, device=DEV).to(torch.bfloat16).requires_grad_()
    g = global_avg_pool_nhwc(x2)
    g2 = x2.detach().float().mean(dim=(1, 2))
    torch.testing.assert_close(g.float(), g2, atol=1e-2, rtol=1e-2)
    dg = torch.randn_like(g)
    g.backward(dg)
    torch.testing.assert_close(x2.grad.float(), (dg.float() / 49)[:, None, None, :].expand_as(x2), atol=1e-3, rtol=1e-2)


@pytest.mark.parametrize("kind", ["sgd", "sgd_nesterov", "adam", "adamw", "rmsprop"])
def test_fused_optimizers_match_cpu_reference(kind):
    from cloud_amd import optim

    torch.manual_seed(3)

    def make(device):
        torch.manual_seed(3)
        m = torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.Linear(65, 7)).to(device)
        m[0].weight.data = m[0].weight.data.to(torch.bfloat16)
        return m

    def opt_for(m):
        if kind == "sgd":
            return optim.SGD(m, learning_rate=0.1, momentum=0.9, weight_decay=1e-2)
        if kind == "sgd_nesterov":
            return optim.SGD(m, learning_rate=0.1, momentum=0.9, nesterov=True)
        if kind == "adam":
            return optim.Adam(m, learning_rate=1e-2, weight_decay=1e-3)
        if kind == "adamw":
            return optim.AdamW(m, learning_rate=1e-2, weight_decay=1e-2)
        return optim.RMSprop(m, learning_rate=1e-2, momentum=0.5)

    mg, mc = make(DEV), make("cpu")
    og, oc = opt_for(mg), opt_for(mc)
    for step in range(4):
        for o in (og, oc):
            for a in o.arenas:
                torch.manual_seed(100 + step)
                a.grad.copy_(torch.randn(a.n).to(a.grad.dtype))
        og.step()
        oc.step()
    for ag, ac in zip(og.arenas, oc.arenas):
        torch.testing.assert_close(ag.master.cpu(), ac.master, atol=1e-5, rtol=1e-5)
        if ag.model is not None:
            torch.testing.assert_close(ag.model.cpu().float(), ac.model.float(), atol=1e-2, rtol=1e-2)


def test_resnet_small_trains_on_gpu():
    from cloud_amd.models.resnet import ResNet
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD

    torch.manual_seed(4)
    m = ResNet((1, 1, 1, 1), num_classes=10, dtype=torch.bfloat16, device=DEV)
    opt = SGD(m, learning_rate=0.05, momentum=0.9)
    x = torch.randn(8, 64, 64, 3, device=DEV).to(torch.bfloat16)
    y = torch.randint(0, 10, (8,), device=DEV)
    losses = []
    for _ in range(15):
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0] * 0.5, losses


@pytest.mark.parametrize("M,K,N", [(1024, 64, 256), (1000, 192, 72), (4096, 256, 64), (512, 2048, 512),
                                   (8, 64, 8), (136, 128, 1000)])
def test_gemm_layouts_vs_fp32(M, K, N):
    from cloud_amd.ops import gemm

    torch.manual_seed(5)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    dy = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    y = gemm.mm_nt(x, w)
    torch.testing.assert_close(y.float(), ref, atol=2e-2 * K ** 0.5, rtol=2e-2)
    dx = gemm.mm_nn(dy, w)
    torch.testing.assert_close(dx.float(), dy.float() @ w.float(), atol=2e-2 * N ** 0.5, rtol=2e-2)
    for splits in (1, 3):
        out32 = torch.zeros(N, K, device=DEV)
        gemm.mm_tn_into(dy, x, out32, beta=0.0, splits=splits)
        torch.testing.assert_close(out32, dy.float().t() @ x.float(), atol=1e-2 * M ** 0.5, rtol=1e-2)
    out16 = torch.ones(N, K, device=DEV).to(torch.bfloat16)
    gemm.mm_tn_into(dy, x, out16, beta=1.0)
    torch.testing.assert_close(out16.float(), 1.0 + dy.float().t() @ x.float(), atol=2e-2 * M ** 0.5, rtol=2e-2)


def test_gemm_stats_epilogue():
    from cloud_amd.ops import gemm

    torch.manual_seed(6)
    M, K, N = 1000, 128, 256
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    tiles = (M + 127) // 128
    stats = torch.zeros(tiles, 2, N, device=DEV)
    y = gemm.mm_nt(x, w, stats=stats)
    yf = y.float()
    torch.testing.assert_close(stats[:, 0].sum(0), yf.sum(0), atol=1e-1, rtol=1e-3)
    torch.testing.assert_close(stats[:, 1].sum(0), (yf * yf).sum(0), atol=1.0, rtol=1e-3)


def test_linear_autograd_writes_arena_grad():
    from cloud_amd.models.layers import Conv2d
    from cloud_amd.optim import SGD

    torch.manual_seed(7)
    conv = Conv2d(64, 128, 1, dtype=torch.bfloat16, device=DEV)
    opt = SGD(conv, learning_rate=0.1)
    x = torch.randn(2, 8, 8, 64, device=DEV).to(torch.bfloat16).requires_grad_()
    y = conv(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    w = conv.weight.detach().float().reshape(128, 64)
    ref_dw = dy.float().reshape(-1, 128).t() @ x.detach().float().reshape(-1, 64)
    torch.testing.assert_close(conv.weight.grad.float().reshape(128, 64), ref_dw, atol=0.5, rtol=2e-2)
    torch.testing.assert_close(x.grad.float().reshape(-1, 64), dy.float().reshape(-1, 128) @ w, atol=0.2, rtol=2e-2)
    # the weight gradient lives inside the optimizer's flat arena, at the slot it was given
    arena = next(a for a in opt.arenas if any(s.param is conv.weight for s in a.slots))
    slot = next(s for s in arena.slots if s.param is conv.weight)
    g = conv.weight.grad
    assert g.untyped_storage().data_ptr() == arena.grad.untyped_storage().data_ptr()
    assert g.data_ptr() == arena.grad.data_ptr() + slot.offset * arena.grad.element_size()
    assert slot.offset + g.numel() <= arena.n


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,p", [
    (2, 14, 64, 64, 3, 1, 1), (2, 15, 64, 128, 3, 2, 1), (2, 16, 8, 64, 7, 2, 3),
    (2, 14, 128, 256, 1, 2, 0), (1, 9, 24, 40, 3, 1, 1), (2, 8, 256, 64, 1, 1, 0),
    # tap-mask loaders: two 64-channel slices per tap, 7x7 maps (every row touches a border),
    # even-sized strided input, 3 images (pixel decode across image boundaries)
    (3, 7, 128, 64, 3, 1, 1), (2, 10, 64, 128, 3, 2, 1), (3, 5, 64, 192, 3, 1, 1),
    # one K tile per kernel row (KW * Cin = 64, stride 1, no padding): the row-segment loader
    (2, 9, 16, 64, 4, 1, 0), (3, 11, 16, 128, 4, 1, 0)])
def test_conv_fwd_dgrad_wgrad_vs_fp32(N, H, Cin, Cout, k, s, p):
    from cloud_amd.ops import conv2d_nhwc

    torch.manual_seed(8)
    x = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(Cout, k, k, Cin, device=DEV) / (k * k * Cin) ** 0.5).to(torch.bfloat16).requires_grad_()
    y = conv2d_nhwc(x, w, None, s, p)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.detach().float().permute(0, 3, 1, 2).requires_grad_()
    yr = F.conv2d(xr, wr, None, s, p).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=5e-2, rtol=3e-2)
    wg = wr.grad.permute(0, 2, 3, 1)
    torch.testing.assert_close(w.grad.float(), wg, atol=3e-2 * wg.abs().max().item() + 1e-2, rtol=3e-2)


def test_conv_stats_partials_feed_bn():
    from cloud_amd.ops import bn_act, conv2d_nhwc

    torch.manual_seed(9)
    x = torch.randn(4, 14, 14, 64, device=DEV).to(torch.bfloat16)
    w = (torch.randn(128, 3, 3, 64, device=DEV) * 0.05).to(torch.bfloat16)
    y, part = conv2d_nhwc(x, w, None, 1, 1, stats=True)
    assert part is not None
    yf = y.float().reshape(-1, 128)
    torch.testing.assert_close(part[:, 0].sum(0), yf.sum(0), atol=1e-1, rtol=1e-3)
    g, b = torch.ones(128, device=DEV), torch.zeros(128, device=DEV)
    out_a = bn_act(y, g, b, torch.zeros(128, device=DEV), torch.ones(128, device=DEV), partials=part)
    out_b = bn_act(y, g, b, torch.zeros(128, device=DEV), torch.ones(128, device=DEV))
    torch.testing.assert_close(out_a.float(), out_b.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("cin,width,stride", [(64, 32, 1), (128, 32, 1), (64, 32, 2)])
def test_fused_bottleneck_matches_fp32_and_unfused(cin, width, stride):
    """Block-level hand-scheduled fwd/bwd (models/fused_block.py) vs the fp32
    PyTorch block and vs the op-by-op autograd path on the same kernels."""
    from cloud_amd.models import fused_block
    from cloud_amd.models.resnet import Bottleneck
    from cloud_amd.optim import SGD

    torch.manual_seed(11)
    blk = Bottleneck(cin, width, stride, dtype=torch.bfloat16, device=DEV, zero_init_residual=False)
    ref = Bottleneck(cin, width, stride, dtype=torch.float32, device=DEV, zero_init_residual=False)
    ref.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in blk.state_dict().items()})
    opt = SGD(blk, learning_rate=0.0)
    x = torch.randn(4, 16, 16, cin, device=DEV).to(torch.bfloat16)
    dy = torch.randn(4, 16 // stride, 16 // stride, 4 * width, device=DEV).to(torch.bfloat16)

    def run(fused):
        blk.fused_block = fused
        opt.zero_grad()
        xi = x.clone().requires_grad_()
        assert fused_block.can_fuse(blk, xi) or not fused
        out = blk(xi)
        out.backward(dy)
        grads = {n: p.grad.detach().float().clone() for n, p in blk.named_parameters()}
        return out.detach().float(), xi.grad.float(), grads

    out_f, dx_f, g_f = run(True)
    out_u, dx_u, g_u = run(False)
    xr = x.float().requires_grad_()
    out_r = ref(xr)
    out_r.backward(dy.float())

    def close(a, b, tol):
        scale = b.abs().max().item() + 1e-3
        torch.testing.assert_close(a, b, atol=tol * scale, rtol=tol)

    def rel(a, b):  # bf16 vs fp32: ReLU masks flip near 0, so compare in norm
        return ((a - b).norm() / (b.norm() + 1e-6)).item()

    assert rel(out_f, out_r.detach()) < 2e-2
    assert rel(dx_f, xr.grad) < 1e-1  # dominated by ReLU-mask flips of near-zero outputs
    close(out_f, out_u, 1e-2)
    close(dx_f, dx_u, 2e-2)
    for n, p in ref.named_parameters():
        assert rel(g_f[n], p.grad.float().reshape(g_f[n].shape)) < 1e-1, n
        close(g_f[n], g_u[n], 2e-2)


def test_native_rccl_communicator_single_rank():
    """The C++ RCCL communicator (world 1 on the one-GPU box): init via unique id,
    side-stream collectives ordered after the compute stream, join before use."""
    from cloud_amd.parallel.comm import RcclComm

    c = RcclComm(rank=0, world=1, device=DEV)
    x = torch.arange(1000, device=DEV, dtype=torch.float32)
    y = x * 2  # produced on the compute stream right before the collective
    c.all_reduce(y)
    c.broadcast(y, root=0)
    out = torch.empty(1000, device=DEV, dtype=torch.float32)
    c.all_gather(out, y)
    rs = torch.empty(1000, device=DEV, dtype=torch.float32)
    c.reduce_scatter(rs, out)
    b = torch.ones(64, device=DEV, dtype=torch.bfloat16)
    c.all_reduce(b)
    c.join()
    assert torch.equal(rs, x * 2) and torch.equal(b, torch.ones_like(b))
    assert c.healthy()
    c.close()


def _relu_bits(mask_bool):
    """[M, C] bool -> the kernels' ReLU bitmask [M, C/8] uint8 (bit j = channel 8c+j)."""
    M, C = mask_bool.shape
    w = (1 << torch.arange(8, device=mask_bool.device)).to(torch.int32)
    return (mask_bool.view(M, C // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


@pytest.mark.parametrize("k,s,p,beta,Cin", [(1, 1, 0, 0.0, 64), (1, 1, 0, 1.0, 64), (3, 1, 1, 0.0, 64),
                                            (3, 2, 1, 0.0, 64), (1, 1, 0, 1.0, 256)])
def test_dgrad_bn_backward_stats_epilogue(k, s, p, beta, Cin):
    """dgrad GEMM epilogue statistics [sum g | sum g*z], g = dx * relu' (fp32 reference),
    and the BN backward fed from them == the BN backward with its own reduction."""
    from cloud_amd.ops import raw

    torch.manual_seed(12)
    N, H, Cout = 3, 15, 128
    OH = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, OH, OH, Cout, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Cout, k, k, Cin, device=DEV) / (k * k * Cin) ** 0.5).to(torch.bfloat16)
    z = (torch.randn(N, H, H, Cin, device=DEV) * 2 + 0.5).to(torch.bfloat16)
    keep = torch.rand(N * H * H, Cin, device=DEV) > 0.4
    bits = _relu_bits(keep)
    base = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16)
    ref = raw.conv_dgrad(dy, w, z.shape, s, p, out=base.clone() if beta else None, beta=beta)
    dx, part = raw.conv_dgrad(dy, w, z.shape, s, p, out=base.clone() if beta else None, beta=beta, bn=(z, bits))
    assert torch.equal(dx, ref)
    g = dx.float().reshape(-1, Cin) * keep
    zf = z.float().reshape(-1, Cin)
    torch.testing.assert_close(part[:, 0].sum(0), g.sum(0), atol=2e-2 * N * H, rtol=1e-3)
    torch.testing.assert_close(part[:, 1].sum(0), (g * zf).sum(0), atol=5e-2 * N * H, rtol=1e-3)

    # BN(+ReLU) backward: partials path vs reduction path (same forward stats)
    gamma, beta_ = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV)
    _, st, mask = raw.bn_fwd(z, gamma, beta_, None, None, 1e-5, 0.1, True, keep_mask=True)
    dg_a, db_a = torch.zeros(Cin, device=DEV), torch.zeros(Cin, device=DEV)
    dg_b, db_b = torch.zeros(Cin, device=DEV), torch.zeros(Cin, device=DEV)
    dx2, part2 = raw.conv_dgrad(dy, w, z.shape, s, p, bn=(z, mask))
    a, _ = raw.bn_bwd(dx2, None, z, gamma, st, True, dgamma=dg_a, dbeta=db_a, mask=mask, partials=part2)
    b, _ = raw.bn_bwd(dx2, None, z, gamma, st, True, dgamma=dg_b, dbeta=db_b, mask=mask)
    torch.testing.assert_close(dg_a, dg_b, atol=1e-2 * N * H, rtol=1e-3)
    torch.testing.assert_close(db_a, db_b, atol=1e-2 * N * H, rtol=1e-3)
    torch.testing.assert_close(a.float(), b.float(), atol=2e-2, rtol=2e-2)


def test_fused_bottleneck_chain_hands_off_bn_statistics(monkeypatch):
    """Consecutive fused blocks: block i+1's conv1 dgrad computes block i's bn3 backward
    statistics (cross-block hand-off) -- and, when block i is a projection block, its
    shortcut BN's statistics too; gradients match the op-by-op path."""
    from cloud_amd.models import fused_block
    from cloud_amd.models.resnet import Bottleneck
    from cloud_amd.ops import raw
    from cloud_amd.optim import SGD

    torch.manual_seed(13)
    net = torch.nn.Sequential(
        Bottleneck(64, 16, 1, dtype=torch.bfloat16, device=DEV, zero_init_residual=False),
        Bottleneck(64, 32, 2, dtype=torch.bfloat16, device=DEV, zero_init_residual=False),
        Bottleneck(128, 32, 1, dtype=torch.bfloat16, device=DEV, zero_init_residual=False))
    opt = SGD(net, learning_rate=0.0)
    x = torch.randn(4, 16, 16, 64, device=DEV).to(torch.bfloat16)
    dy = torch.randn(4, 8, 8, 128, device=DEV).to(torch.bfloat16)
    taken = []
    orig_take = fused_block._take

    def spy(dout):
        r = orig_take(dout)
        taken.append((r[0] is not None, r[1] is not None))
        return r

    monkeypatch.setattr(fused_block, "_take", spy)

    def run(fused, epi):
        monkeypatch.setenv("CLOUD_AMD_BN_BWD_EPILOGUE", "1" if epi else "0")
        for b in net:
            b.fused_block = fused
        opt.zero_grad()
        xi = x.clone().requires_grad_()
        out = net(xi)
        out.backward(dy)
        return xi.grad.float(), {n: p.grad.detach().float().clone() for n, p in net.named_parameters()}

    dx_e, g_e = run(True, True)
    # the last block has no producer; the projection block takes bn3 AND shortcut-BN
    # statistics; the first block takes its bn3 statistics
    assert taken == [(False, False), (True, True), (True, False)], taken
    dx_n, g_n = run(True, False)
    dx_u, g_u = run(False, False)

    def close(a, b, tol=2e-2):
        torch.testing.assert_close(a, b, atol=tol * (b.abs().max().item() + 1e-3), rtol=tol)

    close(dx_e, dx_n)
    close(dx_e, dx_u)
    for n in g_e:
        close(g_e[n], g_n[n])
        close(g_e[n], g_u[n])


def test_stem_space_to_depth_matches_direct_conv():
    """7x7/2/pad3 stem via space-to-depth (4x4/1 over 16 channels): output, BN statistics
    partials and weight gradient equal the direct implicit-GEMM conv on the padded input."""
    from cloud_amd.models.layers import Conv2d
    from cloud_amd.ops import conv as conv_ops

    torch.manual_seed(14)
    conv = Conv2d(8, 64, 7, stride=2, padding=3, dtype=torch.bfloat16, device=DEV)
    x = torch.randn(2, 30, 34, 3, device=DEV).to(torch.bfloat16)
    assert conv_ops.stem_s2d_ok(x, conv.weight, 2, 3)
    y1, p1 = conv_ops.stem_conv_s2d(x, conv.weight, stats=True)
    dy = torch.randn_like(y1)
    y1.backward(dy)
    g1 = conv.weight.grad.detach().float().clone()
    conv.weight.grad = None
    y2, p2 = conv(torch.nn.functional.pad(x, (0, 5)), stats=True)
    y2.backward(dy)
    g2 = conv.weight.grad.detach().float()
    torch.testing.assert_close(y1.float(), y2.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(p1.sum(0), p2.sum(0), atol=0.5, rtol=1e-2)
    assert g1[..., 3:].abs().max().item() == 0.0
    torch.testing.assert_close(g1[..., :3], g2[..., :3], atol=3e-2 * g2.abs().max().item(), rtol=3e-2)


def test_device_loader_normalizes_on_copy_stream(tmp_path):
    """cloud_amd.data.DeviceLoader: pinned slot -> GPU on a copy stream, uint8 -> bf16
    normalisation kernel (csrc/kernels/input.hip) == (x - mean) / std in fp32."""
    from cloud_amd.data import DeviceLoader, NpyBatchLoader, write_npy_dataset

    xp, yp = write_npy_dataset(tmp_path / "ds", 40, image_shape=(6, 10, 3), classes=7, seed=2)
    host = NpyBatchLoader([xp, yp], 8, seed=4, rank=0, world=1, slots=3)
    mean, std = (123.7, 116.3, 103.5), (58.4, 57.1, 57.4)
    dev = DeviceLoader(host, device=DEV, mean=mean, std=std)
    ref_host = NpyBatchLoader([xp, yp], 8, seed=4, rank=0, world=1, slots=2)
    refs = []
    for slot, (xb, yb) in ref_host.epoch(0):
        refs.append((xb.clone(), yb.clone()))
        ref_host.release(slot)
    got = list(dev.epoch(0))
    torch.cuda.synchronize()
    assert len(got) == len(refs) == 5
    m = torch.tensor(mean, device=DEV)
    s = torch.tensor(std, device=DEV)
    for (x, y), (xr, yr) in zip(got, refs):
        assert x.dtype == torch.bfloat16 and x.shape == xr.shape
        torch.testing.assert_close(x.float(), (xr.to(DEV).float() - m) / s, atol=2e-2, rtol=1e-2)
        assert torch.equal(y.cpu(), yr)


def test_u8_normalize_odd_sizes():
    from cloud_amd.ops import _ext

    ext = _ext.load(required=True)
    for n in (3, 48, 51, 4099 * 3):
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=DEV)
        y = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        ext.u8_normalize(x.data_ptr(), y.data_ptr(), n, [10.0, 20.0, 30.0], [2.0, 4.0, 8.0],
                         torch.cuda.current_stream().cuda_stream)
        c = torch.arange(n, device=DEV) % 3
        ref = (x.float() - torch.tensor([10.0, 20.0, 30.0], device=DEV)[c]) / torch.tensor([2.0, 4.0, 8.0],
                                                                                            device=DEV)[c]
        torch.testing.assert_close(y.float(), ref, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("with_bn", [False, True])
def test_dgrad_gated_residual_epilogue(with_bn):
    """1x1 dgrad with res=(src, mask): dx = dgrad + relu'(mask) * src in one epilogue
    (identity-block residual gradient never materialised), with and without the
    BN-backward statistics of dx."""
    from cloud_amd.ops import raw

    torch.manual_seed(15)
    N, H, Cin, Cout = 2, 14, 256, 64
    dy = torch.randn(N, H, H, Cout, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Cout, 1, 1, Cin, device=DEV) / 8).to(torch.bfloat16)
    src = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16)
    keep = torch.rand(N * H * H, Cin, device=DEV) > 0.5
    bits = _relu_bits(keep)
    base = raw.conv_dgrad(dy, w, src.shape, 1, 0)
    ref = base.float() + (src.float().reshape(-1, Cin) * keep).reshape(src.shape)
    if with_bn:
        z = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16)
        zkeep = torch.rand(N * H * H, Cin, device=DEV) > 0.3
        dx, part = raw.conv_dgrad(dy, w, src.shape, 1, 0, beta=1.0, bn=(z, _relu_bits(zkeep)), res=(src, bits))
        g = dx.float().reshape(-1, Cin) * zkeep
        torch.testing.assert_close(part[:, 0].sum(0), g.sum(0), atol=5e-2 * N * H, rtol=1e-3)
        torch.testing.assert_close(part[:, 1].sum(0), (g * z.float().reshape(-1, Cin)).sum(0), atol=1e-1 * N * H,
                                   rtol=1e-3)
    else:
        dx = raw.conv_dgrad(dy, w, src.shape, 1, 0, beta=1.0, res=(src, bits))
    torch.testing.assert_close(dx.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("H,with_bn", [(16, True), (15, True), (14, False)])
def test_sparse_shortcut_dgrad_then_sparse_beta_accumulate(H, with_bn):
    """Projection-block input gradient without the zero-fill: the strided 1x1 shortcut's
    dgrad writes only its non-empty parity class (skip_empty; the other pixels hold NaN
    here) and conv1's 1x1 dgrad accumulates into it reading those pixels as zeros
    (beta_stride).  Must equal the dense pair bitwise, and the fp32 reference closely."""
    from cloud_amd.ops import raw

    torch.manual_seed(21)
    N, Cin, Cd, C1, s = 3, 64, 256, 128, 2
    OH = (H - 1) // s + 1
    dzd = torch.randn(N, OH, OH, Cd, device=DEV).to(torch.bfloat16)
    wd = (torch.randn(Cd, 1, 1, Cin, device=DEV) / Cd ** 0.5).to(torch.bfloat16)
    dz1 = torch.randn(N, H, H, C1, device=DEV).to(torch.bfloat16)
    w1 = (torch.randn(C1, 1, 1, Cin, device=DEV) / C1 ** 0.5).to(torch.bfloat16)
    z = (torch.randn(N, H, H, Cin, device=DEV) + 0.3).to(torch.bfloat16)
    bits = _relu_bits(torch.rand(N * H * H, Cin, device=DEV) > 0.4)
    bn = (z, bits) if with_bn else None

    dense = raw.conv_dgrad(dzd, wd, (N, H, H, Cin), s, 0)
    r_dense = raw.conv_dgrad(dz1, w1, (N, H, H, Cin), 1, 0, out=dense, beta=1.0, bn=bn)
    dx_sp = torch.full((N, H, H, Cin), float("nan"), device=DEV, dtype=torch.bfloat16)
    raw.conv_dgrad(dzd, wd, (N, H, H, Cin), s, 0, out=dx_sp, skip_empty=True)
    even = torch.zeros(H, H, dtype=torch.bool, device=DEV)
    even[::s, ::s] = True
    assert torch.isnan(dx_sp[:, ~even]).all() and not torch.isnan(dx_sp[:, even]).any()
    r_sp = raw.conv_dgrad(dz1, w1, (N, H, H, Cin), 1, 0, out=dx_sp, beta=1.0, bn=bn, beta_stride=s)
    if with_bn:
        assert torch.equal(r_sp[0], r_dense[0])
        torch.testing.assert_close(r_sp[1], r_dense[1], atol=0, rtol=0)
    else:
        assert torch.equal(r_sp, r_dense)
    ref = dz1.float().reshape(-1, C1) @ w1.float().reshape(C1, Cin)
    ref = ref.reshape(N, H, H, Cin)
    ref[:, ::s, ::s] += (dzd.float().reshape(-1, Cd) @ wd.float().reshape(Cd, Cin)).reshape(N, OH, OH, Cin)
    torch.testing.assert_close(dx_sp.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("H,Cd,Cin", [(16, 512, 256), (15, 1024, 512)])
def test_strided_shortcut_dgrad_with_folded_bn_backward(H, Cd, Cin):
    """Projection shortcut input gradient with its BN backward in the operand fetch
    (raw.conv1x1_strided_dgrad_bnbwd): the written dz equals the stride-1 transform-A kernel's
    bitwise, dx's even-even pixels equal that kernel's product bitwise (same tiles, same K
    order), the other pixels stay unwritten, and the result matches an fp32 reference."""
    from cloud_amd.ops import raw

    torch.manual_seed(31)
    N, s = 3, 2
    Ho = (H - 1) // s + 1
    dy = torch.randn(N, Ho, Ho, Cd, device=DEV).to(torch.bfloat16)
    z = torch.randn(N, Ho, Ho, Cd, device=DEV).to(torch.bfloat16)
    keep = torch.rand(N * Ho * Ho, Cd, device=DEV) > 0.4
    bits = _relu_bits(keep)
    coef = torch.randn(3 * Cd, device=DEV) * torch.tensor([1.0, 0.1, 0.01], device=DEV).repeat_interleave(Cd)
    w = (torch.randn(Cd, 1, 1, Cin, device=DEV) / Cd ** 0.5).to(torch.bfloat16)
    side = torch.empty_like(z)
    dx = raw.conv1x1_strided_dgrad_bnbwd(dy, z, bits, coef, w, side, (N, H, H, Cin), s)
    side1 = torch.empty_like(z)
    dx1 = raw.conv1x1_dgrad_bnbwd(dy, z, bits, coef, w, side1)
    torch.cuda.synchronize()
    assert torch.equal(side, side1)
    assert torch.equal(dx[:, ::s, ::s], dx1)
    A, B, D = coef[:Cd], coef[Cd:2 * Cd], coef[2 * Cd:]
    dz = (A * dy.float().reshape(-1, Cd) * keep + B * z.float().reshape(-1, Cd) + D).to(torch.bfloat16).float()
    ref = (dz @ w.float().reshape(Cd, Cin)).reshape(N, Ho, Ho, Cin)
    torch.testing.assert_close(dx[:, ::s, ::s].float(), ref, atol=3e-2, rtol=3e-2)
