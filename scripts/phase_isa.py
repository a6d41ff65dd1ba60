"""Static instruction counts of one step kernel per timed phase, from the assembly of an
HG_TIMING=1 build (the s_memtime / s_memrealtime stamps delimit the phases of DESIGN.md §3).

usage: python scripts/phase_isa.py file.s [kernel-name-filter] [-v SEG]
Counts are static (cold branches included), so they bound the dynamic counts from above.
"""
import collections
import re
import sys


def main():
    text = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else "ILi0ELb0ELb1ELb0ELb0ELb1E"
    show = int(sys.argv[sys.argv.index("-v") + 1]) if "-v" in sys.argv else None
    m = re.search(r"^(_Z\S*step_kernel" + re.escape(filt) + r"\S*):", text, re.M)
    body = text[m.end():text.index(".Lfunc_end", m.end())]
    seg = 0
    cls = collections.defaultdict(collections.Counter)
    ops = collections.defaultdict(collections.Counter)
    for line in body.split("\n"):
        t = line.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op in ("s_memtime", "s_memrealtime"):
            seg += 1
            continue
        kind = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "mem"
        cls[seg][kind] += 1
        ops[seg][op] += 1
    for k in sorted(cls):
        c = cls[k]
        print(f"seg {k:2d}  valu {c['valu']:4d}  salu {c['salu']:4d}  mem {c['mem']:3d}")
    if show is not None:
        for op, n in ops[show].most_common():
            print(f"   {op:28s} {n}")


if __name__ == "__main__":
    main()
