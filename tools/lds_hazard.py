"""Static check of the asm LDS reads in a gfx950 assembly listing (hipcc -S).

The kernels issue ds_read through inline asm and publish the results with their own
`s_waitcnt lgkmcnt` waits, so the compiler treats the destination registers as
written at once.  Any instruction it places between such a read and the wait that
covers it and that reads or writes those registers (a copy on a branch edge, say)
works on the old contents.  This scans each kernel in layout order and reports such
uses; waits retire reads in issue order (lgkmcnt(N) keeps the N youngest pending).

usage: python tools/lds_hazard.py /tmp/mlp_dev.s [kernel-substring]
"""

import re
import sys

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")


def regs(operand_text):
    out = set()
    for m in REG.finditer(operand_text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            for r in range(int(m.group(4)), int(m.group(5)) + 1):
                out.add((m.group(3), r))
    return out


def split_ops(line):
    parts = line.split(None, 1)
    if len(parts) < 2:
        return parts[0], []
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1].split(";")[0])]
    return parts[0], ops


def scan(lines, name):
    in_asm = False
    pending = []  # [(regs, line_no)] in issue order
    hazards = 0
    for no, raw in lines:
        line = raw.strip()
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not line or line.startswith(";") or line.endswith(":"):
            continue
        op, ops = split_ops(line)
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", line)
            if m:
                n = int(m.group(1))
                pending = pending[len(pending) - n:] if n else []
            continue
        if op.startswith("s_endpgm"):
            pending = []
            continue
        is_lds_read = op.startswith("ds_read")
        srcs = set()
        dsts = set()
        if ops:
            if op.startswith(("ds_write", "buffer_store", "global_store", "v_cmp", "s_", "buffer_load")) and \
                    not op.startswith("ds_read"):
                for o in ops:
                    srcs |= regs(o)
                if op.startswith("buffer_load") and "lds" not in line:
                    dsts = regs(ops[0])
                    srcs -= dsts
            else:
                dsts = regs(ops[0])
                for o in ops[1:]:
                    srcs |= regs(o)
        pend_regs = set().union(*[p[0] for p in pending]) if pending else set()
        bad = (srcs | (dsts if not is_lds_read else set())) & pend_regs
        if bad and not (in_asm and line.startswith("s_waitcnt")):
            hazards += 1
            src_line = [p[1] for p in pending if p[0] & bad]
            print(f"{name}: line {no}: '{line}' touches {sorted(bad)[:4]} still pending from line(s) {src_line[:3]}")
        if is_lds_read:
            pending.append((dsts, no))
        elif op.startswith("ds_") or op.startswith("s_load") or op.startswith("s_buffer_load"):
            pending.append((set(), no))
    return hazards


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "pipe_kernel"
    text = open(path).read().split("\n")
    starts = [i for i, x in enumerate(text) if re.match(r"^_Z\w+:", x)]
    total = 0
    for si, s in enumerate(starts):
        name = text[s].split(":")[0]
        if want not in name:
            continue
        e = starts[si + 1] if si + 1 < len(starts) else len(text)
        total += scan([(i + 1, text[i]) for i in range(s, e)], name[:60])
    print(f"{total} hazard(s)")
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
