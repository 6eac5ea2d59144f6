"""Linear-scan waitcnt checker for one AMDGPU asm function: flags a VGPR / SGPR
read (or overwrite) while a load into it may still be outstanding.  Approximate: ignores control flow,
so flags at branch joins need a look at the listing.  usage: waitcnt_check.py <function.s>"""
import re, sys

def regs(tok):
    out = set()
    for m in re.finditer(r'\b([vs])\[(\d+):(\d+)\]|\b([vs])(\d+)\b', tok):
        if m.group(1):
            for i in range(int(m.group(2)), int(m.group(3)) + 1): out.add(f"{m.group(1)}{i}")
        else:
            out.add(f"{m.group(4)}{m.group(5)}")
    return out

lines = open(sys.argv[1]).read().split('\n')
vm = []    # list of (dest regs, line) in order
lgkm = []  # list of (kind, dest regs, line)
for no, l in enumerate(lines, 1):
    s = l.split(';')[0].strip()
    if not s or s.endswith(':') or s.startswith('.'):
        continue
    op = s.split()[0]
    args = s[len(op):].strip()
    parts = [p.strip() for p in args.split(',')] if args else []
    if op == 's_waitcnt':
        m = re.search(r'vmcnt\((\d+)\)', args)
        if m:
            n = int(m.group(1)); vm = vm[len(vm) - n:] if n else []
        m = re.search(r'lgkmcnt\((\d+)\)', args)
        if m:
            n = int(m.group(1))
            if n == 0 or any(k == 's' for k, _, _ in lgkm):
                if n == 0: lgkm = []
                else:
                    # SMEM out of order: only LDS ordering can be assumed
                    lds = [x for x in lgkm if x[0] == 'd']
                    keep = lds[len(lds) - n:]
                    lgkm = [x for x in lgkm if x[0] == 's'] + keep
            else:
                lgkm = lgkm[len(lgkm) - n:]
        continue
    srcs = set()
    dst = set()
    if parts:
        if op.startswith(('global_store', 'buffer_store', 'ds_write', 'scratch_store', 'flat_store', 's_cmp', 's_cbranch', 'global_load_lds', 's_barrier', 'ds_bpermute_b32x')) or op.startswith('s_waitcnt'):
            srcs = set().union(*[regs(p) for p in parts])
        else:
            dst = regs(parts[0]); srcs = set().union(*[regs(p) for p in parts[1:]]) if len(parts) > 1 else set()
    pend_vm = {r: ln for d, ln in vm for r in d}
    pend_lg = {r: ln for _, d, ln in lgkm for r in d}
    for r in srcs | dst:
        if r in pend_vm: print(f"{no}: {s}   <- {r} VMEM load at {pend_vm[r]} outstanding")
        if r in pend_lg: print(f"{no}: {s}   <- {r} LGKM load at {pend_lg[r]} outstanding")
    if op.startswith(('global_load', 'buffer_load', 'scratch_load', 'flat_load')) and not op.startswith('global_load_lds'):
        vm.append((regs(parts[0]), no))
    elif op.startswith('global_load_lds'):
        vm.append((set(), no))
    elif op.startswith(('global_store', 'buffer_store', 'scratch_store')):
        pass
    elif op.startswith('ds_') and not op.startswith(('ds_write', 'ds_swizzle_nop')):
        lgkm.append(('d', regs(parts[0]) if parts else set(), no))
    elif op.startswith('ds_write'):
        lgkm.append(('d', set(), no))
    elif op.startswith('s_load') or op.startswith('s_buffer_load'):
        lgkm.append(('s', regs(parts[0]), no))
