"""Flags VGPRs that a vector-memory instruction reads (address / store data)
and that a later instruction rewrites before the next s_waitcnt vmcnt in
straight-line order (gfx950 reads those operands late; such a rewrite stalls
the wave until the memory op reaches the head of the queue).
usage: python tools/vmem_reg_hazard.py kernel.s"""
import re
import sys


def regs(tok):
    tok = tok.strip().rstrip(",")
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


lines = [l.strip() for l in open(sys.argv[1]) if l.strip() and not l.strip().startswith((";", "."))]
issues = 0
for i, l in enumerate(lines):
    op = l.split()[0]
    if not (op.startswith("global_store") or op.startswith("global_load_lds") or op.startswith("buffer_store")):
        continue
    ops = [t for t in re.split(r",\s*", l[len(op):].strip())]
    read = set()
    for t in ops[:2]:
        read |= regs(t.split()[0] if t else "")
    for j in range(i + 1, len(lines)):
        m = lines[j]
        mop = m.split()[0]
        if mop == "s_waitcnt" and "vmcnt" in m:
            break
        if mop.startswith(("v_", "ds_read", "global_load", "buffer_load")) and not mop.startswith("global_load_lds"):
            dst = m[len(mop):].strip().split(",")[0]
            hit = regs(dst) & read
            if hit:
                issues += 1
                print(f"line {i}: {l}\n   rewritten at {j}: {m}")
                break
print("issues:", issues)
