#!/usr/bin/env python3
"""Print the ISA of one kernel from a --save-temps .s: kasm.py <file.s> <name-substring>"""
import sys
lines = open(sys.argv[1]).read().splitlines()
out, on = [], False
for ln in lines:
    if not on and ':' in ln and sys.argv[2] in ln.split(':')[0] and ln[:1] not in ('.', '\t', ' ', ';'):
        on = True
    if on:
        out.append(ln)
        if 's_endpgm' in ln:
            break
print('\n'.join(out))
