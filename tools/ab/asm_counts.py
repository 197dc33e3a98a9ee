"""Instruction mix per kernel of a hipcc --save-temps gfx950 assembly file.
usage: asm_counts.py FILE.s [substring...]"""
import collections
import re
import subprocess
import sys

s = open(sys.argv[1]).read()
subs = sys.argv[2:]
parts = re.split(r'\n(_Z\w+):[^\n]*\n', s)
for i in range(1, len(parts), 2):
    name = subprocess.run(['c++filt', parts[i]], capture_output=True, text=True).stdout.strip()
    name = name.replace('(anonymous namespace)::', '').split('(')[0]
    if subs and not any(x in name for x in subs):
        continue
    body = parts[i + 1].split('.Lfunc_end')[0]
    c = collections.Counter(re.findall(r'\n\s+([sv]_\w+|ds_\w+|buffer_\w+|global_\w+)', body))
    tot = sum(c.values())
    print('%s: %d instructions' % (name, tot))
    groups = collections.OrderedDict([('ds', 'ds_'), ('f64', '_f64'), ('pk_f32', 'v_pk_'), ('mfma', 'v_mfma'),
                                      ('buffer/global', ('buffer_', 'global_')), ('barrier', 's_barrier'),
                                      ('waitcnt', 's_waitcnt')])
    for g, pat in groups.items():
        pats = pat if isinstance(pat, tuple) else (pat,)
        ks = {k: v for k, v in c.items() if any(p in k for p in pats)}
        if ks:
            print('   %-14s %5d  %s' % (g, sum(ks.values()), ', '.join('%s %d' % kv for kv in sorted(ks.items(), key=lambda x: -x[1])[:6])))
