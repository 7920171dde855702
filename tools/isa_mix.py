#!/usr/bin/env python3
"""Instruction mix per kernel of a hipcc --save-temps .s file: python tools/isa_mix.py file.s"""
import collections
import re
import sys

cur = None
stats = {}
for line in open(sys.argv[1]):
    m = re.match(r'^(_Z\w+):', line)
    if m:
        cur = m.group(1)
        stats[cur] = collections.Counter()
        continue
    if cur is None:
        continue
    t = line.strip()
    if t.startswith('s_endpgm'):
        cur = None
        continue
    if not t or t.startswith(('.', ';')) or ':' in t.split()[0]:
        continue
    op = t.split()[0]
    c = stats[cur]
    c['total'] += 1
    if op.startswith('v_'):
        c['valu'] += 1
        if re.match(r'v_(add|sub|mul|fma|fmac|fmamk|fmaak|max|min)_f32', op):
            c['f32'] += 1
        if 'cndmask' in op:
            c['cndmask'] += 1
    if op.startswith('ds_'):
        c['ds'] += 1
    if op.startswith('s_barrier'):
        c['barrier'] += 1
    if op.startswith(('global_', 'buffer_')):
        c['vmem'] += 1
    if 'dpp' in t:
        c['dpp'] += 1
for k, v in stats.items():
    print(k[:60], dict(v))
