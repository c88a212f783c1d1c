"""Which side of the stem-tail comparison is off: fused vs separate vs fp32 reference."""
import torch
import torch.nn.functional as F

from cloud_amd.models.layers import BatchNormAct, MaxPool2d
from cloud_amd.ops import _ext, gemm, raw
from cloud_amd.ops.pooling import stem_bn_relu_maxpool

_ext.load(required=True)
torch.manual_seed(0)
N, H, W, C = 1, 8, 8, 64
z0 = (torch.randn(N, H, W, C, device="cuda") * 2 + 0.3).to(torch.bfloat16)
M = N * H * W
part = torch.empty(((M + 127) // 128, 2, C), device="cuda")
gemm.fill_stats_torch(z0.view(M, C), part)
bn = BatchNormAct(C, relu=True, device="cuda")
st = raw.bn_fwd_stats(z0, bn.weight, bn.bias, bn.running_mean.clone(), bn.running_var.clone(), 1e-5, 0.1, part)
torch.cuda.synchronize()
zf = z0.float().view(M, C)
mean, var = zf.mean(0), zf.var(0, unbiased=False)
print("mean err", float((st[:C] - mean).abs().max()), "rstd err", float((st[C:2 * C] - torch.rsqrt(var + 1e-5)).abs().max()))
print("scale err", float((st[2 * C:3 * C] - torch.rsqrt(var + 1e-5)).abs().max()),
      "shift err", float((st[3 * C:] + mean * torch.rsqrt(var + 1e-5)).abs().max()))
ya = stem_bn_relu_maxpool(z0.clone(), bn, part)
yb = MaxPool2d(3, 2, 1)(BatchNormAct(C, relu=True, device="cuda")((z0.clone(), part)))
yr = torch.relu((z0.float() - mean) * torch.rsqrt(var + 1e-5))
pre = yr
yr = F.max_pool2d(yr.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
torch.cuda.synchronize()
print("fused vs ref", float((ya.float() - yr).abs().max()), "separate vs ref", float((yb.float() - yr).abs().max()))
for c in range(3):
    print("c", c, "fused", ya[0, :2, :3, c].float().tolist(), "sep", yb[0, :2, :3, c].float().tolist(),
          "ref", yr[0, :2, :3, c].tolist())
print("pre-pool ref ch0 rows0-2", pre[0, :3, :5, 0].tolist())
