"""Instruction mix of k_qp_tiled between s_memtime phase markers (prof build asm)."""
import re
import sys
lines = open(sys.argv[1]).read().split('\n')
start = [i for i, l in enumerate(lines) if re.match(r'^_ZN4kite10k_qp_tiled\S*:', l)][0]
end = [i for i in range(start, len(lines)) if lines[i].strip().startswith('.Lfunc_end')][0]
keys = ['scratch_load', 'scratch_store', 'v_mfma', 'ds_bpermute', 'ds_read', 'ds_write', 'global_load', 's_barrier',
        'v_accvgpr_read', 'v_accvgpr_write', 'v_permlane', '_dpp']
seg, counts = 0, {}
for l in lines[start:end]:
    t = l.strip()
    if t.startswith('s_memtime'):
        seg += 1
    c = counts.setdefault(seg, {'instr': 0})
    if t and not t.startswith(('.', ';')) and not t.endswith(':'):
        c['instr'] += 1
    for k in keys:
        if t.startswith(k) or (k == '_dpp' and '_dpp' in t.split(' ')[0]):
            c[k] = c.get(k, 0) + 1
for s in sorted(counts):
    print(s, counts[s])
