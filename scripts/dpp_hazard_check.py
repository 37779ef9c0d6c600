import re,sys
lines=[l.strip() for l in open(sys.argv[1])]
ins=[l for l in lines if l and not l.startswith((';','.')) and not l.endswith(':')]
def regs(tok):
    m=re.match(r'v\[(\d+):(\d+)\]',tok)
    if m: return set(range(int(m.group(1)),int(m.group(2))+1))
    m=re.match(r'v(\d+)$',tok)
    if m: return {int(m.group(1))}
    return set()
bad=0
for i,l in enumerate(ins):
    if '_dpp' in l.split()[0]:
        src=l.split()[2].rstrip(',')
        r=regs(src)
        ws=0
        for j in range(i-1, max(i-4,-1), -1):
            p=ins[j]; op=p.split()[0]
            if op=='s_nop':
                ws+=int(p.split()[1])+1; continue
            if op.startswith('v_'):
                d=p.split()[1].rstrip(',')
                if regs(d)&r and ws<2:
                    bad+=1; print('HAZARD', i, ins[j], '->', l)
                    break
            ws+=1
            if ws>=2: break
print('dpp hazards:', bad)
