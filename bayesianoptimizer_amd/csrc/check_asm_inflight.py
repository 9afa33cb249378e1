"""Build check: no compiler-generated instruction may touch a register that an inline-asm load is
still filling.

The hand-placed k loops (gpx_trmm_asm.h) issue their ds_read / buffer_load as asm statements whose destination is an
"=v" output and complete them with a later asm s_waitcnt that names the same registers "+v".  That is only correct if
hipcc never reads, copies, moves or reuses those registers in between, which the compiler cannot see: a v_mov of a
fragment register before the wait (hipcc inserts such copies when two control-flow paths meet) reads garbage and
silently corrupts the product (round 6 met exactly that in a TRTRI variant; tools/probes/trtri_blocks.py located it).

This script scans the device assembly that hipcc writes with -save-temps=obj.  Inside ;;#ASMSTART / ;;#ASMEND regions
it tracks the destination registers of ds_read* (lgkmcnt queue) and buffer_load / global_load (vmcnt queue) in issue
order; every s_waitcnt (asm or compiler) retires the oldest entries down to its count.  Any instruction OUTSIDE the
asm regions that names one of the registers still in flight is reported, and the build fails.  The scan is linear in
the file (labels and branches keep the state), which is exact for the straight-line hand-placed sequences it guards.

  python3 check_asm_inflight.py file.s [file.s ...]
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
WAIT_LGKM = re.compile(r"lgkmcnt\((\d+)\)")
WAIT_VM = re.compile(r"vmcnt\((\d+)\)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan(path):
    bad = []
    func = None
    in_asm = False
    lgkm, vm = [], []  # issue-ordered queues of destination-register sets (empty set: no tracked destination)

    def inflight():
        s = set()
        for q in (lgkm, vm):
            for e in q:
                s |= e
        return s

    with open(path) as fh:
        for lineno, raw in enumerate(fh, 1):
            line = raw.strip()
            if line.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if line.startswith(";;#ASMEND"):
                in_asm = False
                continue
            code = line.split(";", 1)[0].strip()
            if not code:
                continue
            if code.endswith(":") and not code.startswith("."):
                if not code.startswith(".L") and not code.startswith("$"):
                    func = code[:-1]
                    lgkm.clear()
                    vm.clear()
                continue
            if code.startswith("."):
                if code.startswith(".Lfunc_end"):
                    lgkm.clear()
                    vm.clear()
                continue
            op, _, args = code.partition(" ")
            args = args.strip()
            if op == "s_waitcnt":
                m = WAIT_LGKM.search(args)
                if m:
                    del lgkm[: max(0, len(lgkm) - int(m.group(1)))]
                m = WAIT_VM.search(args)
                if m:
                    del vm[: max(0, len(vm) - int(m.group(1)))]
                continue
            dst = args.split(",", 1)[0]
            if not in_asm:
                touched = regs(args) & inflight()
                if touched:
                    bad.append((path, lineno, func, code, sorted(touched)[:6]))
            # the queues count every memory operation (asm or not); only asm loads carry tracked registers
            if op.startswith("ds_"):
                lgkm.append(regs(dst) if in_asm and op.startswith("ds_read") else set())
            elif op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime")):
                lgkm.append(set())
            elif op.startswith(("buffer_", "global_", "flat_")):
                vm.append(regs(dst) if in_asm and "load" in op else set())
    return bad


def main(paths):
    bad = []
    for p in paths:
        bad += scan(p)
    for path, lineno, func, code, touched in bad[:40]:
        print(f"{path}:{lineno}: {func}: compiler instruction touches in-flight asm load registers v{touched}: {code}")
    if bad:
        print(f"check_asm_inflight: {len(bad)} violation(s)")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
