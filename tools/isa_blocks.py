"""Per-basic-block instruction counts of one kernel in a hipcc -S listing.
usage: python tools/isa_blocks.py k.s [kernel-substring] [min-count]"""
import re
import sys

src, want = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "rhp_dfa_kernelILi16")
lo = int(sys.argv[3]) if len(sys.argv) > 3 else 12
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"_Z\S*:", l) and want in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].strip() == "s_endpgm")
blocks, cur, cnt = [], ("entry", ""), {}
for l in lines[start:end]:
    t = l.strip()
    if re.match(r"\.LBB\d+_\d+:", t):
        blocks.append((cur, cnt))
        cur, cnt = (t.split(":")[0], t.split(";", 1)[1].strip() if ";" in t else ""), {}
    elif t and not t.startswith((";", ".")) and not t.endswith(":"):
        op = t.split()[0]
        cnt[op] = cnt.get(op, 0) + 1
blocks.append((cur, cnt))
total = 0
for (name, cm), c in blocks:
    n = sum(c.values())
    total += n
    if n >= lo:
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        top = ", ".join(f"{k}:{v}" for k, v in sorted(c.items(), key=lambda x: -x[1])[:5])
        print(f"{name:10s} {n:4d} valu {valu:4d}  {cm[:34]:34s} {top}")
print("total", total)
