"""configs[2] timing: the Gatys loop (VGG-19 up to conv5_1, 5 Gram style layers + relu4_2 content,
Adam) at 512x512 for 300 steps on one MI355X.  Prints one JSON line: ms per step, TFLOP/s of the
algorithmic conv + Gram work (forward and input-gradient convs: 2*cin*cout*9 per output pixel each;
Grams 2*c^2*hw; Gram gradients 2*c^2*hw), the loss at step 0 and at the end and the loss trajectory (every
step's losses recorded on the device inside the timed loop, reported every 10 steps)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import synthetic  # noqa: E402
from neuralstyletransferv1_amd.gatys import Gatys  # noqa: E402

H = W = int(os.environ.get("GATYS_HW", "512"))
STEPS = int(os.environ.get("GATYS_STEPS", "300"))
dev = torch.device("cuda", 0)
sd = synthetic.make_vgg19_state_dict(0)
g = Gatys(sd, dev)
c = (torch.from_numpy(synthetic.make_frames(1, H, W, seed=301)).permute(0, 3, 1, 2).float() / 255).contiguous().to(dev)
s = (torch.from_numpy(synthetic.make_frames(1, H, W, seed=302)).permute(0, 3, 1, 2).float() / 255).contiguous().to(dev)
g.run(c, s, steps=3)  # warm-up
torch.cuda.synchronize()
t0 = time.perf_counter()
x, hist = g.run(c, s, steps=STEPS, trajectory=True)  # every step's losses kept on the device
torch.cuda.synchronize()
dt = time.perf_counter() - t0
convs = ((3, 64, 1), (64, 64, 1), (64, 128, 4), (128, 128, 4), (128, 256, 16), (256, 256, 16), (256, 256, 16),
         (256, 256, 16), (256, 512, 64), (512, 512, 64), (512, 512, 64), (512, 512, 64), (512, 512, 256))
flop = 0
for cin, cout, div in convs:
    flop += 2 * 2 * cin * cout * 9 * (H * W // div)  # forward + input gradient
for cc, div in ((64, 1), (128, 4), (256, 16), (512, 64), (512, 256)):
    flop += 2 * (2 * cc * cc * (H * W // div))  # Gram + its gradient GEMM
ms = dt / STEPS * 1e3
print(json.dumps({"workload": f"configs[2]: Gatys VGG-19 {W}x{H}, {STEPS} Adam steps, bf16 activations / fp32 accumulate",
                  "ms_per_step": round(ms, 3), "steps_per_s": round(STEPS / dt, 2), "total_s": round(dt, 3),
                  "gflop_per_step": round(flop / 1e9, 1), "achieved_tflops": round(flop / (ms * 1e-3) / 1e12, 1),
                  "loss_first": hist[0][1] if hist else None,
                  "loss_last": hist[-1][1] if hist else None,
                  # (step, total, content, style) every 10 steps and the last: the optimisation's trajectory
                  "loss_trajectory": [[h[0]] + [float(f"{v:.6g}") for v in h[1:]] for h in hist
                                      if h[0] % 10 == 0 or h[0] == len(hist) - 1]}), flush=True)
