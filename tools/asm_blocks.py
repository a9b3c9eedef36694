"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (MFMA, LDS, AGPR moves, scratch, VALU)."""
import re, sys
lines = open(sys.argv[1]).read().split('\n')
blocks, cur, name = [], [], 'entry'
for l in lines:
    if re.match(r'^\.LBB\d+_\d+:', l):
        blocks.append((name, cur)); name, cur = l.split(':')[0] + (' LOOP' if 'Loop Header' in l else ''), []
    elif l.startswith('\t') and not l.startswith('\t.') and not l.strip().startswith(';'):
        cur.append(l.strip())
blocks.append((name, cur))
minm = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tot = {}
for n, ins in blocks:
    c = dict(n=len(ins), mfma=sum('v_mfma' in i for i in ins), ard=sum('v_accvgpr_read' in i for i in ins),
             awr=sum('v_accvgpr_write' in i for i in ins), scr=sum(i.startswith('scratch_') for i in ins),
             ds=sum(i.startswith('ds_') for i in ins), glds=sum('global_load_lds' in i for i in ins),
             bar=sum(i.startswith('s_barrier') for i in ins), valu=sum(i.startswith('v_') and 'mfma' not in i and 'accvgpr' not in i for i in ins))
    for k, v in c.items(): tot[k] = tot.get(k, 0) + v
    if c['mfma'] >= minm:
        print(f"{n:22s} " + ' '.join(f"{k}={v}" for k, v in c.items()))
print('TOTAL', tot)
