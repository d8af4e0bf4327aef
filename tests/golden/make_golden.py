"""Generate tests/golden/*.npz from the REFERENCE modules (run in the build container only;
/root/reference does not exist on the GPU box and nothing at test time reads it).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [arch ...]   (only those model cases)

For each architecture the reference class itself (transformer_net.py / transformer_net_nst.py /
model.py, imported from /root/reference) is instantiated, loaded with the seeded synthetic
checkpoint (neuralstyletransferv1_amd/synthetic.py, numpy PCG64) via load_state_dict, and run
on seeded inputs.  Stored: input x, output y, seed, and a sha256 of the weights so a drifting
generator is detected.  Gram vectors come from the reference's utils.gram_matrix.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("NST_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from neuralstyletransferv1_amd import synthetic  # noqa: E402

CASES = [
    # arch, seed, n, h, w, input kind
    ("johnson", 0, 1, 64, 64, "imagenet_255"),
    ("johnson", 1, 2, 96, 128, "raw_255"),
    ("johnson", 2, 1, 50, 70, "raw_255"),      # h,w not divisible by 4 -> output 52x72
    ("nst", 0, 1, 64, 64, "raw_01"),
    ("nst", 1, 1, 72, 100, "raw_01"),
    ("reconet", 0, 1, 64, 64, "imagenet_01"),
    ("reconet", 1, 1, 48, 84, "tanh"),
    ("reconet_frn", 0, 1, 64, 64, "imagenet_01"),   # ReCoNet(frn=True): FRN + TLU (frn.py)
    ("reconet_frn", 1, 2, 48, 84, "tanh"),
]


def weights_sha(sd) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.numpy().tobytes())
    return h.hexdigest()


def ref_module(arch):
    sys.path.insert(0, REF)
    try:
        if arch == "johnson":
            import transformer_net as m
            return m.TransformerNet()
        if arch == "nst":
            import transformer_net_nst as m
            return m.TransformerNet()
        import model as m
        return m.ReCoNet(frn=arch == "reconet_frn")
    finally:
        sys.path.remove(REF)


def encode_for(x01: torch.Tensor, preset: str) -> torch.Tensor:
    # the pipeline.py:1445-1486 encodes, so model inputs have realistic ranges
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    if preset == "imagenet_255":
        return (x01 * 255.0 - mean * 255.0) / (std * 255.0)
    if preset == "imagenet_01":
        return (x01 - mean) / std
    if preset == "tanh":
        return x01 * 2.0 - 1.0
    if preset == "raw_01":
        return x01
    return x01 * 255.0


def main(only=()):
    torch.set_num_threads(8)
    for arch, seed, n, h, w, preset in CASES:
        if only and arch not in only:
            continue
        sd = synthetic.make_state_dict(arch, seed)
        net = ref_module(arch)
        missing, unexpected = net.load_state_dict(sd, strict=False)
        assert not missing and not unexpected, (missing, unexpected)
        net.eval()
        frames = synthetic.make_frames(n, h, w, seed=100 + seed)
        x01 = torch.from_numpy(frames).permute(0, 3, 1, 2).float().div(255)
        x = encode_for(x01, preset).contiguous()
        with torch.no_grad():
            y = net(x)
        path = os.path.join(HERE, f"model_{arch}_s{seed}_{h}x{w}.npz")
        np.savez_compressed(path, x=x.numpy(), y=y.numpy(), frames=frames, seed=seed, preset=preset,
                            weights_sha=weights_sha(sd), torch_version=torch.__version__)
        print(f"{path}: x{tuple(x.shape)} -> y{tuple(y.shape)} range [{float(y.min()):.3f}, {float(y.max()):.3f}]")
    if only:
        return

    sys.path.insert(0, REF)
    import utils as ref_utils
    sys.path.remove(REF)
    g = torch.Generator().manual_seed(7)
    Fm = torch.randn(2, 48, 16, 24, generator=g)
    G = ref_utils.gram_matrix(Fm)
    np.savez_compressed(os.path.join(HERE, "gram_2x48x16x24.npz"), F=Fm.numpy(), G=G.numpy())
    print("gram ok", tuple(G.shape))

    # the reference CLI's flag names (pipeline.py:2157-2410), for the CLI-parity test
    import json
    import re
    src = open(os.path.join(REF, "pipeline.py")).read()
    flags = sorted(set(re.findall(r'add_argument\(\s*"(--[A-Za-z0-9_-]+)"', src)))
    with open(os.path.join(HERE, "reference_flags.json"), "w") as f:
        json.dump({"source": "pipeline.py:2157-2410 add_argument names (extracted by tests/golden/make_golden.py)",
                   "flags": flags}, f, indent=0)
    # mask fixtures: copies of the reference's own input/masks data files
    import shutil
    os.makedirs(os.path.join(HERE, "masks"), exist_ok=True)
    for m in ("center_circle.png", "gradient_horizontal.png"):
        shutil.copyfile(os.path.join(REF, "input", "masks", m), os.path.join(HERE, "masks", m))


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
