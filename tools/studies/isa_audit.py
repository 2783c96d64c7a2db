"""ISA audit of one kernel in a hipcc -S assembly file (round 5):
its register allocation (.vgpr_count / .agpr_count / accum_offset) against every
register the inline asm names, compiler AGPR moves, scratch, and M0 writes outside
inline asm.

  hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S probit_fwd.hip -o fwd.s
  python tools/studies/isa_audit.py fwd.s <mangled kernel name>
"""
import re, sys, collections
s=open(sys.argv[1]).read()
name=sys.argv[2]
i=re.search(re.escape(name)+r':[^\n]*\n', s).end()
j=s.index('.Lfunc_end',i)
body=s[i:j]
blocks = s.split('  - .agpr_count:')
for b in blocks[1:]:
    if '.name:           '+name in b:
        print('agpr_count', b.split('\n')[0].strip(), re.search(r"\.vgpr_count:\s+(\d+)", b).group(1), 'sgpr', re.search(r"\.sgpr_count:\s+(\d+)", b).group(1), 'lds', re.search(r"\.group_segment_fixed_size:\s+(\d+)", b).group(1))
kd=s[s.index('.amdhsa_kernel '+name):]
kd=kd[:kd.index('.end_amdhsa_kernel')]
for k in ('accum_offset','next_free_vgpr','next_free_sgpr'):
    m=re.search(r'\.amdhsa_'+k+r'\s+(\d+)', kd); print(k, m.group(1) if m else None)
used=set(int(x) for x in re.findall(r'\bv(\d+)\b', body))
for a,b2 in re.findall(r'v\[(\d+):(\d+)\]', body):
    used |= set(range(int(a), int(b2)+1))
print('max VGPR index in the kernel body:', max(used))
asms=re.findall(r';;#ASMSTART\n(.*?);;#ASMEND', body, re.S)
c=collections.Counter(); maxv=-1; agpr=False
for a in asms:
    for line in a.strip().split('\n'):
        line=line.strip()
        if not line: continue
        c[line.split()[0]]+=1
        for a1,b1,v1 in re.findall(r'v\[(\d+):(\d+)\]|v(\d+)\b', line):
            maxv=max(maxv,int(b1 or v1))
        if re.search(r'\ba\[?\d', line): agpr=True
print('inline asm statements:', len(asms), dict(c))
print('max VGPR index named by inline asm:', maxv, '| AGPR named by inline asm:', agpr)
print('compiler v_accvgpr ops:', len(re.findall(r'v_accvgpr', body)), '| scratch ops:', len(re.findall(r'\bscratch_', body)))
print('m0 writes outside asm:', len(re.findall(r's_mov_b32 m0', re.sub(r';;#ASMSTART.*?;;#ASMEND', '', body, flags=re.S))))
