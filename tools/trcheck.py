#!/usr/bin/env python3
"""Register hazards of untracked asm LDS reads (ds_read_b64_tr_b16 issued through
inline asm, retired by explicit s_waitcnt lgkmcnt): the compiler treats an asm
result as written when the asm executes, so between the read and the wait that
retires it no instruction may read its registers (stale data) or write them (the
read lands later and overwrites the write).  Walks the kernel's control-flow
graph from a gfx950 assembly listing (hipcc --cuda-device-only -S) with the
in-flight reads as an ordered list (lgkmcnt(k) keeps the newest k; joins take
the element-wise union) and prints every such access.

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S csrc/conv_x3.hip -o /tmp/cx3.s
    python tools/trcheck.py /tmp/cx3.s _ZN3hkp20wgrad_x3_halo_kernelENS_8WgX3ArgsE
"""
import re
import sys


def regs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return frozenset(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return frozenset({int(m.group(1))}) if m else frozenset()


def main():
    path, name = sys.argv[1], sys.argv[2]
    s = open(path).read()
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    lines = [ln.split(';')[0].strip() for ln in s[i:j].split('\n')[1:]]
    blocks, labels, cur = [], {}, []
    for ln in lines:
        m = re.match(r'^(\.LBB\w+):', ln)
        if m:
            blocks.append(cur)
            cur = []
            labels[m.group(1)] = len(blocks)
            continue
        if ln and not ln.startswith('.'):
            cur.append(ln)
            if ln.split()[0].startswith('s_cbranch'):     # a conditional branch ends its block
                blocks.append(cur)
                cur = []
    blocks.append(cur)
    succ = []
    for b, ins in enumerate(blocks):
        out = []
        last = ins[-1] if ins else ''
        for ln in ins:
            op = ln.split()[0]
            if op.startswith(('s_cbranch', 's_branch')):
                out.append(labels[ln.split()[1]])
        if not last.startswith(('s_branch', 's_endpgm')) and b + 1 < len(blocks):
            out.append(b + 1)
        succ.append(out)

    def merge(a, b):
        n = max(len(a), len(b))
        a = [frozenset()] * (n - len(a)) + list(a)
        b = [frozenset()] * (n - len(b)) + list(b)
        return tuple(x | y for x, y in zip(a, b))

    state = {0: ()}
    origin = {}
    work = [0]
    found = set()
    while work:
        b = work.pop()
        st = list(state[b])
        for k, ln in enumerate(blocks[b]):
            op = ln.split()[0]
            toks = [t.strip(',') for t in ln.split()[1:]]
            if op == 's_waitcnt':
                m = re.search(r'lgkmcnt\((\d+)\)', ln)
                if m:
                    n = int(m.group(1))
                    st = st[-n:] if n else []
                continue
            live = frozenset().union(*st) if st else frozenset()
            if op.startswith('ds_read') and 'tr_b16' in op:
                st.append(regs(toks[0]))
                origin.setdefault(regs(toks[0]), set()).add((b, k))
                continue
            if not live:
                continue
            writes = op.startswith('v_') or (op.startswith(('global_load', 'buffer_load', 'ds_read'))
                                             and 'lds' not in op)
            srcs = toks[1:] if writes else toks
            def src_of(rr):
                return sorted(o for rs in st if rs & rr for o in origin.get(rs, ()))[:3]
            if writes and toks and regs(toks[0]) & live:
                found.add(('WRITE', b, k, ln + '   <- read at %s' % src_of(regs(toks[0]))))
            for t in srcs:
                if regs(t) & live:
                    found.add(('READ', b, k, ln + '   <- read at %s' % src_of(regs(t))))
        st = tuple(st)
        for nb in succ[b]:
            new = merge(state[nb], st) if nb in state else st
            if state.get(nb) != new:
                state[nb] = new
                work.append(nb)
    for f in sorted(found, key=lambda x: (x[1], x[2])):
        print('%-5s block %d +%d: %s' % f)
    print('hazards:', len(found))


if __name__ == '__main__':
    main()
