"""Instruction mix of the MFMA loops in a hipcc -save-temps .s file (dev tool)."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
funcs = re.split(r'\n(?=_Z\S+:)', s)
for f in funcs:
    m = re.match(r'(\S+):', f)
    if not m or pat not in m.group(1):
        continue
    lines = [l.split(';')[0].strip() for l in f.split('\n')]
    idx = {}
    for i, l in enumerate(lines):
        mm = re.match(r'^(\.LBB\d+_\d+):', l)
        if mm:
            idx[mm.group(1)] = i
    for i, l in enumerate(lines):
        mm = re.match(r's_cbranch_\w+\s+(\.LBB\d+_\d+)', l)
        if mm and mm.group(1) in idx and idx[mm.group(1)] < i:
            body = [x for x in lines[idx[mm.group(1)]:i + 1] if x and not x.startswith('.')]
            nm = sum('v_mfma' in x for x in body)
            if not nm:
                continue
            c = lambda p: sum(1 for x in body if x.startswith(p))
            print(m.group(1)[20:110], f"loop {mm.group(1)}: mfma {nm} valu {c('v_') - nm} ds {c('ds_')} "
                  f"vmem {c('global_') + c('buffer_')} salu {c('s_')} total {len(body)}")
