"""Instruction mix of one kernel in an ISA dump (hipcc -S): per basic block with >= N of a marker
instruction, the VALU / LDS counts and the opcode histogram.
Usage: python scripts/isa_mix.py <file.s> <kernel-symbol-substring> [marker=v_dot2] [min=4]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
sym, marker = sys.argv[2], (sys.argv[3] if len(sys.argv) > 3 else "v_dot2")
mn = int(sys.argv[4]) if len(sys.argv) > 4 else 4
start = [m.start() for m in re.finditer(r"^(\S+):", s, re.M) if sym in m.group(1)][0]
end = s.index(".Lfunc_end", start)
blocks, cur, name = [], [], "entry"
for l in s[start:end].split("\n"):
    if re.match(r"^\.LBB|^; %bb", l):
        blocks.append((name, cur))
        cur, name = [], l.split()[0] if l.startswith(".") else l.split()[1]
    else:
        cur.append(l.strip())
blocks.append((name, cur))
tot = 0
for n, b in blocks:
    nv = sum(1 for x in b if x.startswith("v_"))
    tot += nv
    if sum(1 for x in b if x.startswith(marker)) >= mn:
        c = Counter(x.split()[0] for x in b if x.startswith("v_"))
        print(n, marker, sum(1 for x in b if x.startswith(marker)), "VALU", nv, "ds",
              sum(1 for x in b if x.startswith("ds_")), "salu",
              sum(1 for x in b if x.startswith("s_") and not x.startswith(("s_waitcnt", "s_nop"))))
        print("   ", sorted(c.items(), key=lambda t: -t[1]))
print("total VALU in kernel", tot)
