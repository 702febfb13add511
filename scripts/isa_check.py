"""Per-kernel ISA census of an amdgcn .s file: AGPR copies, scratch, MFMAs.

usage: python scripts/isa_check.py /tmp/score.s k_score_1p
"""
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
i = 0
while i < len(lines):
    m = re.match(r"^(_Z\S*" + pat + r"\S*):", lines[i])
    if not m:
        i += 1
        continue
    name, body = m.group(1), []
    i += 1
    while i < len(lines) and not lines[i].startswith(".Lfunc_end"):
        body.append(lines[i].strip())
        i += 1
    cnt = lambda op: sum(1 for l in body if l.startswith(op))
    print(f"{name[:70]:70s} agpr_w={cnt('v_accvgpr_write')} agpr_r={cnt('v_accvgpr_read')} "
          f"agpr_mov={cnt('v_accvgpr_mov')} scratch={cnt('scratch_')} mfma={cnt('v_mfma')} "
          f"vmcnt0={sum(1 for l in body if 'vmcnt(0)' in l)}")
