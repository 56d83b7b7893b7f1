"""Rough VGPR liveness over a straight-line stretch of gfx950 assembly (diagnostics only).

Usage: python tools/vgpr_live.py file.s START END [TOP]
Backward scan from END to START treating the code as straight-line (branches ignored): reports
the TOP lines with the most live VGPRs. Defs are the first operand of VALU / load / MFMA
instructions; stores, ds_write and s_* instructions define no VGPR."""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok):
    out = []
    for m in REG.finditer(tok):
        if m.group(1):
            out += list(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.append(int(m.group(3)))
    return out


def main():
    path, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 15
    lines = open(path).read().split("\n")
    live = set()
    rows = []
    for ln in range(b, a - 1, -1):
        t = lines[ln - 1].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":") or t.startswith("s_"):
            rows.append((len(live), ln, t))
            continue
        op, _, rest = t.partition(" ")
        ops = [x.strip() for x in rest.split(",")]
        nodef = op.startswith(("global_store", "scratch_store", "ds_write", "buffer_store", "ds_add", "ds_bpermute"))
        if op.startswith("ds_bpermute"):
            nodef = False
        defs = [] if nodef or not ops else regs(ops[0])
        uses = []
        for x in (ops if nodef else ops[1:]):
            uses += regs(x)
        if op.startswith("v_mfma") and len(ops) >= 4:
            uses += regs(ops[3])  # the accumulator input
        for r in defs:
            live.discard(r)
        for r in uses:
            live.add(r)
        rows.append((len(live), ln, t))
    rows.sort(reverse=True)
    for n, ln, t in rows[:top]:
        print(n, ln, t[:80])


if __name__ == "__main__":
    main()


def live_at(path, a, b, at):
    """Live VGPRs just before line `at` (backward scan from b), with each one's defining line."""
    lines = open(path).read().split("\n")
    live = set()
    for ln in range(b, at - 1, -1):
        t = lines[ln - 1].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":") or t.startswith("s_"):
            continue
        op, _, rest = t.partition(" ")
        ops = [x.strip() for x in rest.split(",")]
        nodef = op.startswith(("global_store", "scratch_store", "ds_write", "buffer_store", "ds_add"))
        defs = [] if nodef or not ops else regs(ops[0])
        uses = []
        for x in (ops if nodef else ops[1:]):
            uses += regs(x)
        if op.startswith("v_mfma") and len(ops) >= 4:
            uses += regs(ops[3])
        for r in defs:
            live.discard(r)
        for r in uses:
            live.add(r)
    defl = {}
    for ln in range(a, at):
        t = lines[ln - 1].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":") or t.startswith("s_"):
            continue
        op, _, rest = t.partition(" ")
        ops = [x.strip() for x in rest.split(",")]
        if op.startswith(("global_store", "scratch_store", "ds_write", "buffer_store", "ds_add")) or not ops:
            continue
        for r in regs(ops[0]):
            defl[r] = (ln, op)
    return sorted(live), defl
