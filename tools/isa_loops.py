#!/usr/bin/env python3
"""ISA accounting of a kernel's loops (round 5): split one function of a
hipcc -S listing into basic blocks, find the loops (a branch back to an
earlier label), and count each loop body's instructions by class:
VALU, SALU (split into branch / exec-mask / wait / nop / readlane-spill /
address+other), LDS, VMEM, SMEM.  Usage:
    isa_loops.py listing.s symbol-substring [--dump N]
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith(('ds_',)):
        return 'LDS'
    if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')):
        return 'VMEM'
    if op.startswith('s_load') or op.startswith('s_buffer_load'):
        return 'SMEM'
    if op in ('v_readlane_b32', 'v_writelane_b32', 'v_readfirstlane_b32'):
        return 'V_LANE'
    if op.startswith('v_'):
        return 'VALU'
    if op.startswith('s_waitcnt'):
        return 'S_WAIT'
    if op == 's_barrier':
        return 'S_BARRIER'
    if op.startswith('s_nop'):
        return 'S_NOP'
    if op.startswith('s_cbranch') or op == 's_branch' or op.startswith('s_setpc'):
        return 'S_BRANCH'
    if 'saveexec' in op or op.startswith('s_andn2_b64') or op.startswith('s_or_b64') \
            or op.startswith('s_and_b64') or op.startswith('s_xor_b64') or op.startswith('s_mov_b64'):
        return 'S_MASK64'
    if op.startswith('s_cmp') or op.startswith('s_cselect') or op.startswith('s_bitcmp'):
        return 'S_CMP'
    if op.startswith('s_'):
        return 'S_OTHER'
    return 'OTHER'


def load(path, sym):
    lines = open(path).read().split('\n')
    start = None
    for i, l in enumerate(lines):
        if l.startswith('_Z') and sym in l.split(':')[0] and l.split(';')[0].rstrip().endswith(':'):
            start = i
            break
    if start is None:
        sys.exit('symbol not found')
    body = []
    for l in lines[start + 1:]:
        if l.startswith('.Lfunc_end'):
            break
        body.append(l)
    return lines[start].split(':')[0], body


def blocks(body):
    blk = OrderedDict()
    cur = '<entry>'
    blk[cur] = []
    for l in body:
        s = l.strip()
        m = re.match(r'^(\.LBB\w+):', s)
        if m:
            cur = m.group(1)
            blk[cur] = []
            continue
        if not s or s.startswith(';') or s.startswith('.'):
            continue
        blk[cur].append(s.split(';')[0].strip())
    return blk


def main():
    path, sym = sys.argv[1], sys.argv[2]
    dump = int(sys.argv[sys.argv.index('--dump') + 1]) if '--dump' in sys.argv else 0
    name, body = load(path, sym)
    blk = blocks(body)
    names = list(blk)
    idx = {n: i for i, n in enumerate(names)}
    print(name)
    tot = Counter(classify(i.split()[0]) for b in blk.values() for i in b)
    print('function:', sum(len(b) for b in blk.values()), 'instructions', dict(tot))
    loops = []
    for n, ins in blk.items():
        for i in ins:
            op = i.split()[0]
            if op.startswith('s_cbranch') or op == 's_branch':
                tgt = i.split()[-1]
                if tgt in idx and idx[tgt] <= idx[n]:
                    loops.append((tgt, n))
    for (h, t) in loops:
        seg = names[idx[h]:idx[t] + 1]
        ins = [i for s in seg for i in blk[s]]
        c = Counter(classify(i.split()[0]) for i in ins)
        nb = c['S_BARRIER']
        print(f'\nloop {h} .. {t}: {len(seg)} blocks, {len(ins)} instructions, {nb} barriers')
        steps = max(nb // 2, 1)
        for k in sorted(c):
            print(f'  {k:10s} {c[k]:6d}  per step {c[k] / steps:7.1f}')
        ops = Counter(i.split()[0] for i in ins)
        sal = [(o, k) for o, k in ops.most_common() if o.startswith('s_')]
        print('  top SALU ops:', sal[:25])
        val = [(o, k) for o, k in ops.most_common() if o.startswith('v_')]
        print('  top VALU ops:', val[:25])
        if dump and len(ins) >= dump:
            for s in seg:
                print(s + ':')
                for i in blk[s]:
                    print('    ' + i)


if __name__ == '__main__':
    main()
