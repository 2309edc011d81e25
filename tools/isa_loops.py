"""Per-loop instruction census of a kernel in hipcc -save-temps / --cuda-device-only -S
output: python tools/isa_loops.py <file.s> <mangled kernel name prefix>. Prints every
loop (a label with a backward branch to it) holding >= 20 DPP FMAs (round 5)."""
import re, sys
lines=open(sys.argv[1]).read().split('\n')
fn=sys.argv[2]
start=next(i for i,l in enumerate(lines) if l.startswith(fn))
end=next(i for i in range(start,len(lines)) if 's_endpgm' in lines[i])
body=lines[start:end+1]
labels={}
for i,l in enumerate(body):
    m=re.match(r'^(\.LBB\d+_\d+):',l)
    if m: labels[m.group(1)]=i
pats={'dpp':'v_fmac_f64_dpp','ds_read':'ds_read','gl_lds':'global_load_lds','bufst':'buffer_store','f64':r'v_(add|fma|mul|fmac)_f64(?!_dpp)','salu':r'^\s+s_(?!waitcnt|nop)','vmov':'v_mov|v_cndmask','wait':'s_waitcnt','nop':'s_nop','perm':'permlane|bpermute|v_readlane|readfirstlane'}
for i,l in enumerate(body):
    m=re.search(r's_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)',l)
    if not m: continue
    tgt=m.group(1) or m.group(2)
    if tgt not in labels or labels[tgt] >= i: continue
    a=labels[tgt]
    ins=[s for s in body[a:i+1] if s.startswith('\t') and not s.strip().startswith((';','.'))]
    c={k:sum(1 for s in ins if re.search(p,s)) for k,p in pats.items()}
    if c['dpp']>=20:
        print(tgt, f"lines {a}-{i}", "insts", len(ins), c)
