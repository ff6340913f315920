"""Per basic block instruction counts of an ISA dump (hipcc -S), for blocks with >= N v_fma_f64.
Usage: python scripts/isa_blocks.py <file.s> [min_fma]"""
import re, sys
s = open(sys.argv[1]).read().split('\n'); mn = int(sys.argv[2]) if len(sys.argv) > 2 else 16
blocks, cur, name = [], [], 'entry'
for l in s:
    if re.match(r'^\.LBB|^; %bb', l):
        blocks.append((name, cur)); cur = []; name = l.split()[0] if l.startswith('.') else l.split()[1]
    else:
        cur.append(l.strip())
blocks.append((name, cur))
for n, b in blocks:
    nf = sum(1 for x in b if x.startswith('v_fma_f64'))
    if nf >= mn:
        nv = sum(1 for x in b if x.startswith('v_'))
        print(n, 'fma', nf, 'VALU', nv, 'ds', sum(1 for x in b if x.startswith('ds_')),
              'salu', sum(1 for x in b if x.startswith('s_') and not x.startswith(('s_waitcnt', 's_nop'))),
              'nop', sum(1 for x in b if x.startswith('s_nop')))
