"""Write the synthetic checkpoints of every architecture as the flat files tools/asan/nst_asan_driver reads
(int32 arch, int32 count, then per tensor: int32 name length, name bytes, int64 numel, float32 data)."""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from neuralstyletransferv1_amd import _lib, synthetic  # noqa: E402

ARCHS = {"johnson": _lib.NST_ARCH_JOHNSON, "nst": _lib.NST_ARCH_NST, "reconet": _lib.NST_ARCH_RECONET,
         "reconet_frn": _lib.NST_ARCH_RECONET_FRN}


def main(out_dir=HERE):
    paths = []
    for name, arch in ARCHS.items():
        sd = synthetic.make_state_dict(name, 0)
        path = os.path.join(out_dir, f"params_{name}.bin")
        with open(path, "wb") as f:
            f.write(struct.pack("<ii", arch, len(sd)))
            for k, v in sd.items():
                a = np.ascontiguousarray(v.detach().cpu().float().numpy().reshape(-1))
                kb = k.encode()
                f.write(struct.pack("<i", len(kb)) + kb + struct.pack("<q", a.size))
                f.write(a.astype("<f4").tobytes())
        paths.append(path)
    return paths


if __name__ == "__main__":
    print("\n".join(main()))
