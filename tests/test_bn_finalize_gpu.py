"""BatchNorm statistics finalize from GEMM-epilogue partials (csrc/kernels/bn.hip
group_finalize_kernel): the group reduction and the per-channel finalize run as ONE launch --
the last block of each 64-channel column block (agent-scope ticket) sums the group rows in a
fixed order and finalizes.  Checked against fp64 PyTorch sums of the same partials, repeated
(the ticket words must re-arm), on a second stream, bitwise-stable across repeats, for channel
counts of 1 to 32 column blocks."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _partials(z, rows=128):
    M, C = z.shape
    return z.reshape(M // rows, rows, C)


@pytest.mark.parametrize("C,tiles", [(64, 3000), (256, 25088), (2048, 400)])
def test_forward_finalize_matches_fp64(C, tiles):
    from cloud_amd.ops import raw

    torch.manual_seed(C)
    z = (torch.randn(tiles * 128, C, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    zf = _partials(z.float())
    part = torch.stack([zf.sum(1), (zf * zf).sum(1)], 1).contiguous()  # [tiles][2][C]
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda")
    outs = []
    for stream in (torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.current_stream()):
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        with torch.cuda.stream(stream):
            st = raw.bn_fwd_stats(z, gamma, beta, rm, rv, 1e-5, 0.1, part)
        torch.cuda.synchronize()
        outs.append((st.clone(), rm.clone(), rv.clone()))
    M = z.shape[0]
    s = part[:, 0].double().sum(0)
    q = part[:, 1].double().sum(0)
    mean = s / M
    var = (q / M - mean * mean).clamp_min(0)
    rstd = 1 / torch.sqrt(var + 1e-5)
    for st, rm, rv in outs:
        torch.testing.assert_close(st[:C].double(), mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(st[C:2 * C].double(), rstd, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(st[2 * C:3 * C].double(), gamma.double() * rstd, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rm.double(), 0.1 * mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rv.double(), 0.9 + 0.1 * var * M / (M - 1), rtol=1e-5, atol=1e-6)
    for st, rm, rv in outs[1:]:  # fixed summation order: identical whichever block finishes last
        assert torch.equal(st, outs[0][0]) and torch.equal(rm, outs[0][1]) and torch.equal(rv, outs[0][2])


@pytest.mark.parametrize("C,tiles", [(128, 6272), (1024, 1568)])
def test_backward_finalize_matches_fp64(C, tiles):
    from cloud_amd.ops import raw

    torch.manual_seed(7 + C)
    M = tiles * 128
    part = torch.randn(tiles, 2, C, device="cuda") * 10
    mean = torch.randn(C, device="cuda")
    rstd = torch.rand(C, device="cuda") + 0.5
    stats = torch.cat([mean, rstd, torch.zeros(2 * C, device="cuda")])
    gamma = torch.rand(C, device="cuda") + 0.5
    coefs = []
    for _ in range(3):
        dg, db = torch.ones(C, device="cuda"), torch.ones(C, device="cuda")
        coef = raw.bn_bwd_coef(C, M, gamma, stats, part, dgamma=dg, dbeta=db, accumulate=1)
        torch.cuda.synchronize()
        coefs.append(coef.clone())
    sd = part[:, 0].double().sum(0)
    sdx = rstd.double() * (part[:, 1].double().sum(0) - mean.double() * sd)
    k1 = gamma.double() * rstd.double()
    torch.testing.assert_close(dg.double(), 1 + sdx, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(db.double(), 1 + sd, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(coefs[0][:C].double(), k1, rtol=1e-6, atol=1e-7)
    # B and D are differences of sums of +-10 partials (fp32 group sums): judged against their scale
    B = -k1 * (sdx / M) * rstd.double()
    torch.testing.assert_close(coefs[0][C:2 * C].double(), B, rtol=1e-4, atol=1e-4 * float(B.abs().max()))
    D = -k1 * (sd / M) + k1 * (sdx / M) * rstd.double() * mean.double()
    torch.testing.assert_close(coefs[0][2 * C:].double(), D, rtol=1e-4, atol=1e-4 * float(D.abs().max()))
    assert all(torch.equal(c, coefs[0]) for c in coefs[1:])
