"""Static VALU instruction count of one kernel in a .s file (experiment)."""
import sys
s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
ins = [l.strip() for l in s[i:j].splitlines() if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
print(name[:60], 'total', len(ins), 'valu', sum(1 for l in ins if l.startswith('v_')),
      'salu', sum(1 for l in ins if l.startswith('s_')))
