import torch, torch.nn.functional as F, sys
sys.path.insert(0, '.')
from mtl_das_pytorch_amd.ops import functional as fn
C=8; B,H,W=4,9,21
y = (torch.randn(B, C, H, W) * 2 + 0.5).bfloat16().float().cuda()
stats = torch.zeros(8, 2, C, device="cuda", dtype=torch.float64)
stats[0, 0] = y.sum((0, 2, 3)); stats[0, 1] = (y * y).sum((0, 2, 3))
gamma = torch.ones(C, device="cuda"); beta = torch.zeros(C, device="cuda")
rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
nbt = torch.zeros(1, device="cuda", dtype=torch.int64)
bn = fn.bn_args(stats, gamma, beta, rm, rv, nbt, B*H*W)
print(bn)
out = fn.bn_tail(0, y.permute(0,2,3,1).contiguous().bfloat16(), bn)
torch.cuda.synchronize()
print("stats", stats[0])
print("mean", y.mean((0,2,3)), "var", y.var((0,2,3), unbiased=False))
print("rm/0.1", rm/0.1, "rv", rv, "nbt", nbt)
o = out.permute(0,3,1,2).float()
yy = y
# fit out = a*y + b per channel
for c in range(2):
    A = torch.stack([yy[:,c].flatten(), torch.ones_like(yy[:,c].flatten())],1)
    sol = torch.linalg.lstsq(A.cpu(), o[:,c].flatten().unsqueeze(1).cpu()).solution
    print("chan", c, "scale/shift", sol.flatten().tolist())
