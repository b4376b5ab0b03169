"""Instruction mix of the kernels in a hipcc -save-temps .s file: python isa_mix.py file.s [filter]"""
import collections, re, sys
s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
parts = re.split(r'\n([_A-Za-z]\w+):\s*;\s*@', s)
for k in range(1, len(parts), 2):
    name, body = parts[k], parts[k + 1].split('.Lfunc_end')[0]
    if flt not in name:
        continue
    ins = [l.strip().split()[0] for l in body.split('\n')
           if l.strip() and not l.strip().startswith(('.', ';')) and not l.strip().endswith(':')]
    c = collections.Counter(ins)
    valu = sum(v for n, v in c.items() if n.startswith('v_'))
    vg = re.search(r'\.vgpr_count:\s+(\d+)', s[s.find(name + ':'):]) 
    print(f"{name[:90]}  total {len(ins)}  valu {valu}")
    print("   " + ", ".join(f"{n} {v}" for n, v in c.most_common(24)))
