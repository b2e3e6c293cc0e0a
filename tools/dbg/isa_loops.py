"""Instruction mix of the inner loops of one kernel in a hipcc -S listing."""
import re, sys
s = open(sys.argv[1]).read()
pat = sys.argv[2]
names = [m for m in re.findall(r'^(_Z\S+):', s, re.M) if pat in m]
for name in names:
    i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
    k = s[i:j]
    blocks = []; cur = None
    for l in k.split('\n'):
        t = l.strip()
        if re.match(r'^\.LBB\d+_\d+:', t):
            cur = [t, []]; blocks.append(cur)
        elif cur and t and not t.startswith(('.', ';')):
            cur[1].append(t)
    print(name)
    for lab, ins in blocks:
        c = {}
        for x in ins:
            op = x.split()[0]
            key = 'nop' if op == 's_nop' else 'valu' if op.startswith('v_') else 'ds' if op.startswith('ds_') else 'vmem' if op.startswith(('global_', 'buffer_')) else 'wait' if op.startswith('s_waitcnt') else 'salu' if op.startswith('s_') else op
            c[key] = c.get(key, 0) + 1
        if len(ins) > 40: print(' ', lab[:12], len(ins), c)
    ops = {}
    for x in k.split('\n'):
        t = x.strip().split()
        if t and t[0].startswith('v_'): ops[t[0]] = ops.get(t[0], 0) + 1
    print('  top VALU:', sorted(ops.items(), key=lambda a: -a[1])[:14])
