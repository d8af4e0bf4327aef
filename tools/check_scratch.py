"""Build report: scratch use by the kernels whose LDS-DMA loads are waited for with hand-counted
`s_waitcnt vmcnt(N)` (conv_wstat, conv_wphase, conv_ws9, conv_gemm's LDS-DMA kernel) and the other asm-MFMA kernel
(conv_ws2).  Those kernels are meant to
keep everything in registers with their K loops fully unrolled; scratch means spills or a loop the compiler kept
rolled with its accumulators in memory (the Makefile's per-file unroll flag missing: a deconv1 variant ran 6x
slower that way).  Scratch there is not only slow, it is WRONG: the MFMAs of these kernels are inline asm with the
accumulator tied in place (conv_ws_common.h mfma_tied), opaque to hipcc, which therefore does not know an MFMA's
result lands several cycles after issue.  A spill or a rolled loop moves accumulators through scratch right after
the asm, and the scratch store (or a VALU copy) can read the register before the MFMA has written it: the likely
cause of what the round-3 deconv2 probe without the unroll flag recorded (gpurun_out/w4.log: 421159 of 423936
deconv2 outputs wrong, from the first element; the same source with the unroll flag is exact).  The counted vmcnt waits themselves stay safe (an extra vector-memory instruction
only makes a vmcnt(N) wait stricter).  So the build FAILS on any scratch in these files (NST_STRICT_SCRATCH=0
turns it into a report, for experiment builds only).
Reads the compiler's -Rpass-analysis=kernel-resource-usage remarks and echoes every other diagnostic.

    python3 tools/check_scratch.py <remarks file>
"""
import os
import re
import sys


def main(path: str) -> int:
    bad, name, n, in_remark = [], None, 0, False
    for line in open(path, errors="replace"):
        if "kernel-resource-usage" not in line:
            if in_remark and re.match(r"^\s*\d*\s*\|", line):
                continue  # a remark's source-context / caret line
            in_remark = False
            sys.stderr.write(line)  # warnings and errors of the compile itself
            continue
        in_remark = True
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m:
            n += 1
            if int(m.group(1)) > 0:
                bad.append((name, int(m.group(1))))
    if bad:
        for k, s in bad:
            sys.stderr.write(f"check_scratch: {k} uses {s} bytes/lane of scratch (spills in a counted-vmcnt kernel)\n")
        return 0 if os.environ.get("NST_STRICT_SCRATCH") == "0" else 1
    if n == 0:
        sys.stderr.write(f"check_scratch: no kernel-resource-usage remarks in {path}\n")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
