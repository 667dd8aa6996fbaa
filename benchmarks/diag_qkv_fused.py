import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
from collective_communication_mpi_amd import _native
dev = _native.device(); st = torch.cuda.current_stream().cuda_stream
B, S, H, D, kp = 5, 16, 4, 64, 8
HD = H * D
g = torch.Generator(device="cuda").manual_seed(1)
xp = (torch.randn(B * S, kp, device="cuda", generator=g) * 0.5).bfloat16()
w = (torch.randn(3 * HD, kp, device="cuda", generator=g) / kp ** 0.5).bfloat16()
bq = torch.randn(3 * HD, device="cuda", generator=g) * 0.1
wo = torch.zeros(16, HD, device="cuda").bfloat16()
qkv = torch.full((B * S, 3 * HD), float("nan"), device="cuda").bfloat16()
lse = torch.empty(B * H, S, device="cuda"); pool = torch.empty(B, HD, device="cuda", dtype=torch.bfloat16)
z = torch.zeros((B * S, 16), device="cuda"); bo = torch.zeros(16, device="cuda")
dev.attn_qkv_fwd(xq=xp.data_ptr(), ld_xq=xp.stride(0), kq=kp, wq=w.data_ptr(), ld_wq=w.stride(0), bq=bq.data_ptr(),
                 qkv_out=qkv.data_ptr(), ld_qkv=qkv.stride(0), ztok=z.data_ptr(), zrows=0, zpush=[], lse=lse.data_ptr(),
                 B=B, S=S, Hl=H, D=D, scale=D ** -0.5, pool=pool.data_ptr(), ld_pool=pool.stride(0), wo=wo.data_ptr(),
                 ld_wo=wo.stride(0), n_out=16, bo=bo.data_ptr(), ld_zt=16, stream=st)
torch.cuda.synchronize()
ref = (xp.float() @ w.float().T + bq)
got = qkv.float()
torch.set_printoptions(precision=3, linewidth=200, sci_mode=False)
bad = ~torch.isclose(got, ref, rtol=1e-2, atol=1e-2)
print("bad frac", bad.float().mean().item())
v = bad.view(B, S, 3, H, D // 16, 16)
print("by sel", v.float().mean(dim=(0, 1, 3, 4, 5)))
print("by head", v.float().mean(dim=(0, 1, 2, 4, 5)))
print("by nt", v.float().mean(dim=(0, 1, 2, 3, 5)))
print("by token", v.float().mean(dim=(0, 2, 3, 4, 5)))
print("by col c", v.float().mean(dim=(0, 1, 2, 3, 4)))
print("by b", v.float().mean(dim=(1, 2, 3, 4, 5)))
print("got[0,:16]", got[0, :16]); print("ref[0,:16]", ref[0, :16])
print("got[1,:16]", got[1, :16]); print("ref[1,:16]", ref[1, :16])
print("bias only", bq[:16])
print("xw only", (xp.float() @ w.float().T)[0, :16])
