#!/usr/bin/env python3
"""Static check of k_score_1p's AGPR row tiles: no instruction may read a
tile register (v_accvgpr_read / v_accvgpr_mov / an MFMA source) while the
inline-asm load that writes it can still be in flight.

The tile loads are inline asm, so the compiler does not know they are
asynchronous: when it runs short of AGPRs it may copy a freshly "loaded"
register elsewhere before its s_waitcnt — a copy of stale bits (round 4: the
lazy-view variant with HH = 2 at p = 2048 read a[0:3] right after issuing
its load; the first tile of every workgroup scored garbage).

A linear scan per kernel (branches ignored): vector-memory ops are queued in
issue order, `s_waitcnt vmcnt(N)` retires all but the newest N, an AGPR is
in flight from its asm load until retired.

usage: python scripts/tile_hazard_check.py file.s [kernel-substring]
       (file.s: hipcc --offload-arch=gfx950 --cuda-device-only -S ...)
exit status 1 when a hazard is found.
"""
import re
import sys

VMEM = re.compile(r"^(global_|buffer_|scratch_|flat_)(load|store|atomic)")


def regs(tok):
    """AGPR indices named by an operand token (a5, a[4:7])."""
    m = re.fullmatch(r"a(\d+)", tok)
    if m:
        return [int(m.group(1))]
    m = re.fullmatch(r"a\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []


def check(lines, name):
    queue = []  # vector-memory ops in issue order: set of AGPRs each writes (empty for others)
    bad = []
    for n, raw in enumerate(lines):
        l = raw.split(";")[0].strip()
        if not l or l.endswith(":") or l.startswith("."):
            continue
        op = l.split()[0]
        ops = [t.strip() for t in l[len(op):].split(",")]
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", l)
            if m:
                keep = int(m.group(1))
                queue = queue[len(queue) - keep:] if keep < len(queue) else queue
                if keep == 0:
                    queue = []
            continue
        inflight = set().union(*queue) if queue else set()
        if VMEM.match(op):
            srcs = ops[1:] if "load" in op else ops
            for t in srcs:
                if set(regs(t)) & inflight:
                    bad.append((n, l))
            dst = set(regs(ops[0])) if "load" in op else set()
            queue.append(dst)
            continue
        if op.startswith("v_"):
            srcs = ops[1:]
            if op.startswith("v_mfma"):
                srcs = ops[1:]  # A, B, C
            for t in srcs:
                if set(regs(t)) & inflight:
                    bad.append((n, l))
            # a write to an in-flight register would be overwritten by the load
            if set(regs(ops[0])) & inflight and not op.startswith("v_mfma"):
                bad.append((n, l))
    return bad


def main():
    src = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_score_1p"
    lines = open(src).read().split("\n")
    i, nbad, nk = 0, 0, 0
    while i < len(lines):
        m = re.match(r"^(_Z\S*" + pat + r"\S*):", lines[i])
        if not m:
            i += 1
            continue
        name, body = m.group(1), []
        i += 1
        while i < len(lines) and not lines[i].startswith(".Lfunc_end"):
            body.append(lines[i])
            i += 1
        nk += 1
        bad = check(body, name)
        if bad:
            nbad += 1
            print(f"HAZARD {name[:80]}: {len(bad)} reads of in-flight tile registers, first: line {bad[0][0]}: {bad[0][1]}")
    print(f"{nk} kernels checked, {nbad} with hazards")
    return 1 if nbad else 0


if __name__ == "__main__":
    sys.exit(main())
