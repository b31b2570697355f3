"""Static check for the LDS-read hazard of hand-placed inline asm ("LDS hazards").

An inline-asm ds_read is asynchronous: its destination registers are valid only after an s_waitcnt lgkmcnt that
covers it. hipcc does not know that, so a use of the registers can be scheduled between the asm read and a
separate asm s_waitcnt (round 6 hit exactly this in the in-conv GroupNorm: every output NaN). The kernels tie each
result to the wait with an empty asm ("+v"); this checker scans the device assembly for any use of an asm
ds_read_b* destination register before the next s_waitcnt lgkmcnt(0).

    python scripts/lds_asm_check.py file.s     (prints the violations, exit 1 if any)
"""
import re
import sys


def _regs(text):
    out = set(re.findall(r"\bv(\d+)\b", text))
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        out |= {str(r) for r in range(int(a), int(b) + 1)}
    return {int(r) for r in out}


def check(asm_text, window=400):
    """[(function, read line, offending line)] for every asm ds_read whose destination is read before an
    s_waitcnt lgkmcnt(N) that covers it (N <= the LDS operations issued after it: LDS completes in order). Only
    reads emitted from inline asm (between ;;#ASMSTART / ;;#ASMEND) are checked."""
    lines = asm_text.split("\n")
    bad, func, in_asm = [], "?", False
    for n, line in enumerate(lines):
        m = re.match(r"^([A-Za-z_][\w.$]*):", line)
        if m and not line.startswith(".L"):
            func = m.group(1)
        if ";;#ASMSTART" in line:
            in_asm = True
            continue
        if ";;#ASMEND" in line:
            in_asm = False
            continue
        if not in_asm:
            continue
        mm = re.match(r"\s*ds_read\w*\s+(v\[\d+:\d+\]|v\d+)\s*,", line)
        if not mm:
            continue
        dst = _regs(mm.group(1))
        younger = 0      # LDS operations issued after this read (they complete in order)
        for k in range(n + 1, min(len(lines), n + window)):
            t = lines[k].split(";")[0]
            w = re.search(r"lgkmcnt\((\d+)\)", t) if "s_waitcnt" in t else None
            if w and int(w.group(1)) <= younger:
                break    # at most N outstanding and N younger ones exist: this read has completed
            if re.match(r"\s*ds_", t):
                younger += 1
                if re.match(r"\s*ds_read", t):
                    continue
            if not t.strip():
                continue
            ops = t.strip().split(None, 1)
            if len(ops) < 2:
                continue
            # a write of the register (first operand of a VALU op) is not a use; any source operand is
            srcs = ops[1].split(",", 1)[1] if "," in ops[1] else ""
            if ops[0].startswith(("v_", "ds_write", "buffer_", "global_")) and (_regs(srcs) & dst or
                                                                              (ops[0].startswith(("ds_write", "buffer_store", "global_store")) and _regs(ops[1]) & dst)):
                bad.append((func, line.strip(), t.strip()))
                break
    return bad


if __name__ == "__main__":
    v = check(open(sys.argv[1]).read())
    for f, r, u in v:
        print(f"{f}: {r}  used by  {u}")
    sys.exit(1 if v else 0)
