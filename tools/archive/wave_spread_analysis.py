import numpy as np, sys
z=np.load(sys.argv[1])
wid,dur,hw,xcc=z['wid'],z['dur'],z['hw_id'],z['xcc']
m=dur.mean(0)
print("waves",len(wid),"mean",m.mean().round(2),"std of per-wave mean",m.std().round(2),"mean per-launch std",dur.std(1).mean().round(2))
simd=(hw>>4)&3; cu=(hw>>8)&15; sh=(hw>>12)&1; se=(hw>>13)&7
def by(name,key):
    ks=sorted(set(key.tolist())); vals=[m[key==k].mean() for k in ks]
    print(f"{name}: groups {len(ks)}, spread of group means {np.ptp(vals):.2f} µs, std {np.std(vals):.2f}; ", ' '.join(f'{k}:{v:.1f}' for k,v in list(zip(ks,vals))[:40]))
by("simd",simd); by("se",se); by("sh",sh); by("cu",cu)
by("xcc,se",xcc*8+se)
cuid=((xcc*8+se)*2+sh)*16+cu
ks=sorted(set(cuid.tolist())); vals=np.array([m[cuid==k].mean() for k in ks])
print("per-CU means: n",len(ks),"std",vals.std().round(2),"range",vals.min().round(1),vals.max().round(1))
# within-CU spread
w_in=np.mean([m[cuid==k].std() for k in ks]); print("mean within-CU std",round(w_in,2))
by("wid%4",wid%4); by("wid%8",wid%8); by("wid%16",wid%16)
# address-based: byte offset of the wave's K block, mod power-of-two windows
off=wid.astype(np.int64)*4*38400
for gran in (256,4096,65536):
  for nch in (16,32,64,128):
    ch=(off//gran)%nch
    ks=sorted(set(ch.tolist()))
    if len(ks)<2: continue
    vals=[m[ch==k].mean() for k in ks]
    print(f"K-block channel model gran {gran} nch {nch}: groups {len(ks)} std {np.std(vals):.2f}")
