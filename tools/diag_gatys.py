"""Layer-by-layer check of the Gatys backward (scratch diagnostic): dL/dz of each conv, GPU vs torch autograd."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, '.')
from neuralstyletransferv1_amd import synthetic
from neuralstyletransferv1_amd.gatys import Gatys
from oracle import gatys_oracle as GO
from oracle import nst_oracle as O
sd = synthetic.make_vgg19_state_dict(0)
g = Gatys(sd, torch.device("cuda", 0))
H = 128
c = torch.from_numpy(synthetic.make_frames(1, H, H, seed=301)).permute(0, 3, 1, 2).float().div(255).contiguous()
s = torch.from_numpy(synthetic.make_frames(1, H, H, seed=302)).permute(0, 3, 1, 2).float().div(255).contiguous()
x = (0.5 * c + 0.5 * s).contiguous()
g.set_targets(c.cuda(), s.cuda())
lw = [0, 1, 0, 0, 0]
grad, losses, dz = g.grad_capture(x.cuda(), 0.0, 1e6, lw)
# CPU: z of every conv with retain_grad
with torch.no_grad():
    fs = GO.features(sd, s)
A = [O.gram_matrix(fs[i]) for i in GO.STYLE_IDX]
h = (x.clone().requires_grad_(True) - GO.MEAN) / GO.STD
zs = []
for idx, pool in GO.CONVS:
    z = F.conv2d(h, sd[f"features.{idx}.weight"], sd[f"features.{idx}.bias"], padding=1)
    z.retain_grad()
    zs.append(z)
    a = F.relu(z)
    h = F.max_pool2d(a, 2) if pool else a
loss = 0
for k, (i, wl) in enumerate(zip((0, 2, 4, 8, 12), lw)):
    if wl:
        loss = loss + 1e6 * wl * F.mse_loss(O.gram_matrix(F.relu(zs[i])), A[k])
loss.backward()
for i in range(12, -1, -1):
    a = dz[i].float().cpu()
    b = zs[i].grad
    if b is None or float(b.norm()) == 0:
        print(i, "cpu grad zero; gpu norm", float(a.norm()))
        continue
    cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-30))
    print(i, tuple(b.shape), "cos", round(cos, 5), "ratio", round(float(a.norm() / b.norm()), 4), flush=True)
# from the GPU's dz2: CPU conv-transpose (data grad of conv2_1) then max-pool backward with the CPU z1_2
dz2 = dz[2].float().cpu()
gp = torch.nn.grad.conv2d_input((1, 64, H // 2, H // 2), sd["features.5.weight"], dz2, padding=1)
z12 = zs[1].detach()
a12 = F.relu(z12)
for label, zz in (("fp32 z1_2", a12), ("bf16 z1_2", F.relu(z12.to(torch.bfloat16).float()))):
    pooled, idx = F.max_pool2d(zz, 2, return_indices=True)
    gz = F.max_unpool2d(gp, idx, 2, output_size=zz.shape[-2:]) * (z12 > 0)
    a = dz[1].float().cpu()
    cos = float((a * gz).sum() / (a.norm() * gz.norm()))
    print("dz1 from gpu dz2 via CPU bwd,", label, "cos", round(cos, 5), flush=True)
pooled, idx = F.max_pool2d(a12, 2, return_indices=True)
# which windows disagree: GPU dz1 nonzero positions vs CPU argmax
a = dz[1].float().cpu()
nz_gpu = (a != 0)
gzc = F.max_unpool2d(gp, idx, 2, output_size=a12.shape[-2:]) * (z12 > 0)
nz_cpu = (gzc != 0)
print("nonzero gpu", int(nz_gpu.sum()), "cpu", int(nz_cpu.sum()), "both", int((nz_gpu & nz_cpu).sum()), flush=True)
# full bf16 emulation on the CPU: bf16 weights, bf16 normalised input, bf16 stored z (straight-through)
def rb(t):
    return t + (t.to(torch.bfloat16).float() - t).detach()
xr = x.clone().requires_grad_(True)
h = rb((xr - GO.MEAN) / GO.STD)
zs2 = []
for idx, pool in GO.CONVS:
    z = F.conv2d(h, sd[f"features.{idx}.weight"].to(torch.bfloat16).float(), sd[f"features.{idx}.bias"], padding=1)
    z = rb(z)
    z.retain_grad()
    zs2.append(z)
    a = F.relu(z)
    h = F.max_pool2d(a, 2) if pool else a
loss = 1e6 * F.mse_loss(O.gram_matrix(F.relu(zs2[2])), A[1])
loss.backward()
for i in (2, 1, 0):
    a = dz[i].float().cpu()
    b = zs2[i].grad
    cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-30))
    print("bf16-emulated", i, "cos", round(cos, 5), flush=True)
gx = grad.cpu() / GO.STD
cos = float((gx * xr.grad).sum() / (gx.norm() * xr.grad.norm()))
print("bf16-emulated image grad cos", round(cos, 5), flush=True)
