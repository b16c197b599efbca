"""Host emulation of the LRU eviction sweep's two cluster walks ("The eviction
sweep, rebuilt"): k_gc_clusters' interleaved per-slot walk vs k_lru_clusters' mask walk (all
deletions of a 32-slot chunk before its moves; move targets from the home distance in the
occupancy masks of the chunk and the one before, else from the table).  Random linear-probing
tables with 4-slot home groups, tombstones, up to 0.99 load and wrap-around, and a capped
distance (7) to exercise the table fallback.  python tools/lru_walk_emu.py -> "bad 0"."""
import random

EMPTY, FULL, TOMB = 0, 1, 2
def seq(st, home, kill):
    n=len(st); st=st[:]; pos=list(range(n))  # pos: which original entry occupies slot
    ident=list(range(n))
    starts=[i for i in range(n) if st[i]!=EMPTY and st[i-1]==EMPTY]
    for s0 in starts:
        j=s0; hole=False
        while st[j]!=EMPTY:
            if st[j]==TOMB: st[j]=EMPTY; hole=True
            elif kill[ident[j]]: st[j]=EMPTY; hole=True
            elif hole:
                p=home[ident[j]]
                while p!=j:
                    if st[p]==EMPTY:
                        st[p]=FULL; ident[p]=ident[j]; st[j]=EMPTY; break
                    p=(p+1)%n
            j=(j+1)%n
    return [(st[i], ident[i] if st[i]==FULL else None) for i in range(n)]
def masks(st, home, kill, cap=255):
    n=len(st); nw=n//32; orig=st[:]; st=st[:]; ident=list(range(n))
    code_dist=[min((i-home[i])%n, cap) for i in range(n)]
    starts=[i for i in range(n) if orig[i]!=EMPTY and orig[i-1]==EMPTY]
    def mk(cw):
        emp=tmb=kil=0
        for b in range(32):
            x=orig[cw*32+b]
            if x==EMPTY: emp|=1<<b
            elif x==TOMB: tmb|=1<<b
            elif kill[cw*32+b]: kil|=1<<b
        return emp,tmb,kil
    M=0xffffffff
    def ctz(x): return (x & -x).bit_length()-1
    def move(j,p):
        st[p]=FULL; ident[p]=ident[j]; st[j]=EMPTY
    for w in range(nw):
        m=0
        for s0 in starts:
            if s0//32==w: m|=1<<(s0%32)
        if not m: continue
        e0=mk(w)
        while m:
            frm=ctz(m); cw=w; emp,tmb,kil=e0; prev=M; hole=False
            while True:
                rng=(M<<frm)&M; e=emp&rng
                inn= rng & ((1<<ctz(e))-1) if e else rng
                gone=(tmb|kil)&inn
                g=gone
                while g: st[cw*32+ctz(g)]=EMPTY; g&=g-1
                cur=(~emp & ~gone)&M
                mv=inn&~gone
                if not hole: mv = mv & ~((2<<ctz(gone))-1) & M if gone else 0
                while mv:
                    t=ctz(mv); j=cw*32+t
                    dist=code_dist[j] if st[j]==FULL else None
                    # code_dist is per original slot j: the entry at j is the original one (moves only go backwards)
                    dist=code_dist[j]
                    if dist<=32+t and dist<cap:
                        win=(cur<<32)|prev; pj=32+t; ph=pj-dist
                        span=((1<<pj)-1)&~((1<<ph)-1)
                        fr=~win&span
                        if fr:
                            pp=ctz(fr)
                            p= cw*32+pp-32 if pp>=32 else ((cw-1)%nw)*32+pp
                            move(j,p); cur&=~(1<<t)
                            if pp>=32: cur|=1<<(pp-32)
                            else: prev|=1<<pp
                    else:
                        hm=(j-dist)%n if dist<cap else home[j]
                        p=hm
                        while p!=j:
                            if st[p]==EMPTY:
                                move(j,p); cur&=~(1<<t)
                                if p//32==cw: cur|=1<<(p%32)
                                elif p//32==(cw-1)%nw: prev|=1<<(p%32)
                                break
                            p=(p+1)%n
                    mv&=mv-1
                if gone: hole=True
                if e: break
                cw=(cw+1)%nw; emp,tmb,kil=mk(cw); prev=cur; frm=0
            m = 0 if cw!=w else m&(m-1)
    return [(st[i], ident[i] if st[i]==FULL else None) for i in range(n)]
def build(n, load, tombp, seed, homespread):
    r=random.Random(seed); st=[EMPTY]*n; home=[0]*n
    for k in range(int(n*load)):
        h=r.randrange(n)//4*4 if homespread else r.randrange(n)
        p=h
        while st[p]!=EMPTY: p=(p+1)%n
        st[p]=FULL; home[p]=h
    for i in range(n):
        if st[i]==FULL and r.random()<tombp: st[i]=TOMB
    kill=[st[i]==FULL and r.random()<0.2 for i in range(n)]
    return st,home,kill
bad=0
for seed in range(300):
    n=random.Random(seed).choice([64,128,256,1024])
    load=random.Random(seed+1).choice([0.2,0.5,0.8,0.95,0.99])
    st,home,kill=build(n,load,0.05,seed,seed%2)
    if EMPTY not in st: continue
    for cap in (255, 7):
        a=seq(st,home,kill); b=masks(st,home,kill,cap)
        if a!=b: bad+=1; print("MISMATCH", seed, n, load, cap); break
print("bad", bad)
