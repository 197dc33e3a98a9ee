"""Instruction census of one kernel in a hipcc -S output (usage: asm_stats.py file.s substr...)."""
import re
import sys

s = open(sys.argv[1]).read()
for sub in sys.argv[2:]:
    for m in re.finditer(r'^(_Z\S*):\s*;', s, re.M):
        name = m.group(1)
        if sub not in name:
            continue
        start = m.end()
        end = s.index('.Lfunc_end', start)
        body = s[start:end]
        c = lambda pat: len(re.findall(pat, body))
        print('%-44s lines %6d  s_load %4d (x16 %d x8 %d x4 %d x2 %d)  gl_ld %4d gl_st %4d  ds_rd %4d ds_wr %4d  '
              'waitcnt %4d barrier %3d  valu~ %5d  scratch %d' % (
                  name[:44], body.count('\n'), c(r's_load_dword'), c(r's_load_dwordx16'), c(r's_load_dwordx8'),
                  c(r's_load_dwordx4'), c(r's_load_dwordx2 '), c(r'global_load'), c(r'global_store'),
                  c(r'ds_read'), c(r'ds_write'), c(r's_waitcnt'), c('s_barrier'), c(r'\n\s+v_'), c('scratch_')))
