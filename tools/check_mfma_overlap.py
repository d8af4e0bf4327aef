"""Scan gfx950 assembly for MFMAs whose destination registers partially overlap a source A / B register.

hipcc (ROCm 7.2) allocated `v_mfma_f32_16x16x16_f16 v[178:181], v[92:93], v[178:179], v[130:133]` for a builtin
MFMA in conv_ws9.hip's split-weight variant: the B operand lives in the destination's first two registers, and
the result's first two values came out wrong (tools/dbg/f16m_conv1.py: channels 4k, 4k + 1 of one tile row).
This reports every such instruction in an assembly file (hipcc --cuda-device-only -S): PARTIAL overlaps (exit 1)
and, with --all, exact ones (the destination register range equal to a source's: the generic kernels have a few and
are bit-exact in their tests, so the hardware reads the whole operand before it writes).

    python3 tools/check_mfma_overlap.py [--all] <file.s> [...]
"""
import re
import sys

REG = re.compile(r"([va])(?:\[(\d+):(\d+)\]|(\d+))")


def regs(tok):
    m = REG.fullmatch(tok.strip())
    if not m:
        return None
    kind = m.group(1)
    if m.group(4) is not None:
        lo = hi = int(m.group(4))
    else:
        lo, hi = int(m.group(2)), int(m.group(3))
    return kind, lo, hi


def main(paths):
    show_all = "--all" in paths
    paths = [p for p in paths if p != "--all"]
    bad = 0
    for path in paths:
        func = "?"
        for ln, line in enumerate(open(path, errors="replace"), 1):
            if re.match(r"^[_A-Za-z][\w.]*:", line) and not line.startswith("."):
                func = line.split(":")[0]
            s = line.strip()
            if not s.startswith("v_mfma"):
                continue
            ops = [o.strip() for o in s.split(None, 1)[1].split(",")]
            if len(ops) < 3:
                continue
            d, a, b = regs(ops[0]), regs(ops[1]), regs(ops[2])
            for src in (a, b):
                if d and src and d[0] == src[0] and not (src[2] < d[1] or src[1] > d[2]):
                    exact = (src[1], src[2]) == (d[1], d[2])
                    if not exact:
                        bad += 1
                    if show_all or not exact:
                        print(f"{path}:{ln}: {func}: {'exact' if exact else 'PARTIAL'}: {s}")
                    break
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
