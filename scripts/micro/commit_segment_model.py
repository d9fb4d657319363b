# Sequential model of the S commit's per-wave segmented OR (el_gpu.hip commit_s_sorted, step 4):
# 64 lanes emulated, the atomics applied in lane order, 2000 random waves checked against a
# one-candidate-at-a-time reference.  Usage: python3 scripts/micro/commit_segment_model.py
import random
def wave(keys, bits, word_state):
    # keys: list of (x, w) per lane (None = off); bits: bit index per lane
    L=64; NONE=0xffffffff
    on=[k is not None for k in keys]
    m=[(1<<bits[l]) if on[l] else 0 for l in range(L)]
    wx=[keys[l][0] if on[l] else NONE for l in range(L)]
    ww=[keys[l][1] if on[l] else (NONE-l) for l in range(L)]
    up=lambda a,d: [a[l-d] if l>=d else a[l] for l in range(L)]
    down=lambda a,d: [a[l+d] if l+d<L else a[l] for l in range(L)]
    px,pw=up(wx,1),up(ww,1)
    head=[1 if (l==0 or px[l]!=wx[l] or pw[l]!=ww[l]) else 0 for l in range(L)]
    incl=m[:]; f=head[:]
    d=1
    while d<64:
        o,of=up(incl,d),up(f,d)
        ni,nf=incl[:],f[:]
        for l in range(L):
            if l>=d:
                if not f[l]: ni[l]=incl[l]|o[l]
                nf[l]=f[l]|of[l]
        incl,f=ni,nf; d<<=1
    before=up(incl,1)
    excl=[0 if head[l] else before[l] for l in range(L)]
    hd=down(head,1)
    tail=[1 if (l==63 or hd[l]) else 0 for l in range(L)]
    old=[0]*L
    for l in range(L):   # serialized atomics in lane order
        if tail[l] and incl[l]:
            k=(wx[l],ww[l]); old[l]=word_state.get(k,0); word_state[k]=old[l]|incl[l]
    nw=[]
    for l in range(L):
        last=next(j for j in range(l,64) if tail[j])
        seen=old[last]|excl[l]
        nw.append(on[l] and (seen&m[l])==0)
    return nw
random.seed(1)
for trial in range(2000):
    st={}; ref={}
    keys=[]; bits=[]
    for l in range(64):
        if random.random()<0.1: keys.append(None); bits.append(0); continue
        keys.append((random.randint(0,2), random.randint(0,2))); bits.append(random.randint(0,3))
    # sort like the sorted chunk would (adjacent equal words), but allow collisions: random order sometimes
    if trial%2==0:
        idx=sorted(range(64), key=lambda l: (keys[l] is None, keys[l] or (0,0)))
        keys=[keys[i] for i in idx]; bits=[bits[i] for i in idx]
    nw=wave(keys,bits,st)
    # reference: sequential
    for l in range(64):
        if keys[l] is None: 
            assert not nw[l]; continue
        k=keys[l]; b=1<<bits[l]
        new=(ref.get(k,0)&b)==0; ref[k]=ref.get(k,0)|b
        assert new==nw[l], (trial,l)
print("ok")
