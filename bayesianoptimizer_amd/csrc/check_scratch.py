"""Build check (Makefile): no kernel that runs the hand-placed asm k loop of gpx_trmm_asm.h may use scratch memory.

Reads the -Rpass-analysis=kernel-resource-usage remarks of one object and fails (exit 1) when a kernel of the asm-tile
families reports ScratchSize > 0.  Their loads are asm statements whose "=v" outputs must stay in place until the wait
that completes them; a spill or register copy inserted by the compiler in between would read a stale value silently.
Kernels outside these families may spill (moments_grad_kernel's and fps_kernel's per-lane arrays, rocPRIM's sort); their
scratch is reported, not fatal.  Compiler warnings in the remarks file are echoed.
"""
import re
import sys

ASM_TILE_KERNELS = ("trmm_sumsq_kernel", "potrf_step_kernel", "mll_grad_kernel", "svgp_w2_kernel", "trtri_t_kernel",
                    "trtri_w_kernel")


def main(path: str) -> int:
    text = open(path, encoding="utf-8", errors="replace").read()
    for line in text.splitlines():
        if "warning:" in line or "error:" in line:
            print(line)
    bad = []
    name = None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name is not None and int(m.group(1)) > 0:
            if any(k in name for k in ASM_TILE_KERNELS):
                bad.append((name, int(m.group(1))))
    for name, size in bad:
        print(f"{path}: {name} uses {size} bytes/lane of scratch; the hand-placed asm k loop requires none")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
