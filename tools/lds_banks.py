"""LDS bank-conflict model of the backward sweep's Qxx transpose (round 6): extra LDS-array cycles
per wave-instruction for a candidate block layout at(r, c) and problem stride D (in reals), from the
banking table of MI355X_MICROARCH.md ("LDS": lane groups and bank formula per instruction).

  python tools/lds_banks.py        (prints the round-5 row-major and the column-major layouts)
"""
import itertools
def rho_wb(t): return (t>>1) if (t<14 and t%2==0) else (7+(t>>1) if t<14 else t)
def rho_srb(t): return (t>>1) if (t<6 and t%2==0) else (3+(t>>1) if t<6 else t)
# bank conflict extra cycles for one wave instruction; addrs: list of (lane, dword_addr, ndw)
def cost(form, accs):
    # groups & bank modulus
    if form in ("rd64",): groups=[range(0,32),range(32,64)]; mod=64
    elif form=="rd2_64" or form=="wr64" or form=="add64": groups=[range(i,i+16) for i in (0,16,32,48)]; mod=32
    elif form=="rd128": groups=[[*range(0,4),*range(12,16),*range(20,28)],[*range(4,12),*range(16,20),*range(28,32)],
                                 [*range(32,36),*range(44,48),*range(52,60)],[*range(36,44),*range(48,52),*range(60,64)]]; mod=64
    elif form=="wr128": groups=[range(i,i+8) for i in range(0,64,8)]; mod=32
    elif form in ("rd32","wr32","add32"): groups=[range(0,32),range(32,64)]; mod=32
    d=dict((l,(a,n)) for l,a,n in accs)
    extra=0
    for g in groups:
        banks={}
        for l in g:
            if l not in d: continue
            a,n=d[l]
            for k in range(n):
                banks.setdefault((a+k)%mod,set()).add(a+k)
        if banks: extra+=max(len(s) for s in banks.values())-1
    return extra

def eval_layout(at, D, fp=64, rd_forms=("rd64","rd2_64"), wr_forms=("wr64",), filler=None, verbose=False):
    sz = 2 if fp==64 else 1
    res={}
    def A(p,r,c): return sz*(p*D + at(r,c))
    rd = ["rd64","rd2_64"] if fp==64 else ["rd32"]
    wr = ["wr64"] if fp==64 else ["wr32"]
    ad = "add64" if fp==64 else "add32"
    tot={}
    # PAIRS2
    for name,acc in (("p2",None),("r4",None),("srb",None)):
        c_rd={f:0 for f in rd}; c_wr={f:0 for f in wr}; c_ad=0
        if name=="p2":
            for s in range(7):
                w=[];r=[]
                for t in range(64):
                    q=t//32; row=(t//16)%2; tt=t%16; rh=rho_wb(tt)
                    cr = rh if tt<14 else (filler(tt) if filler else rh)
                    w.append((t,A(q,rh,(7 if row else 0)+s),sz))
                    r.append((t,A(q,(7 if row else 0)+s,cr),sz))
                for f in wr: c_wr[f]+=cost(f,w)
                for f in rd: c_rd[f]+=cost(f,r)
            a=[(t,A(t//32,rho_wb(t%16),rho_wb(t%16)),sz) for t in range(64)]
            c_ad=cost(ad,a)
        elif name=="r4":
            for j in range(16):
                w=[(t,A(t//16,rho_wb(t%16),j),sz) for t in range(64)]
                for f in wr: c_wr[f]+=cost(f,w)
            for j in range(14):
                r=[]
                for t in range(64):
                    tt=t%16; rh=rho_wb(tt); cr= rh if tt<14 else (filler(tt) if filler else rh)
                    r.append((t,A(t//16,j,cr),sz))
                for f in rd: c_rd[f]+=cost(f,r)
            a=[(t,A(t//16,rho_wb(t%16),rho_wb(t%16)),sz) for t in range(64)]
            c_ad=cost(ad,a)
        else:
            for j in range(10):
                w=[(t,A(t//16,rho_srb(t%16),j),sz) for t in range(64)]
                for f in wr: c_wr[f]+=cost(f,w)
            for j in range(6):
                r=[]
                for t in range(64):
                    rh=rho_srb(t%16); cr= rh if rh<10 else 0
                    r.append((t,A(t//16,j,cr),sz))
                for f in rd: c_rd[f]+=cost(f,r)
            a=[(t,A(t//16,rho_srb(t%16),rho_srb(t%16)),sz) for t in range(64)]
            c_ad=cost(ad,a)
        tot[name]=(c_wr,c_rd,c_ad)
    return tot

def eval_reads128(at, D):
    # reads of pairs (j, j+1) as one b128 (contiguous in memory)
    tot={}
    def A(p,r,c): return 2*(p*D+at(r,c))
    c=0
    for s in range(0,7,2):
        r=[]
        for t in range(64):
            q=t//32; row=(t//16)%2; tt=t%16; rh=rho_wb(tt)
            r.append((t,A(q,(7 if row else 0)+s,rh),4))
        c+=cost("rd128",r)
    tot['p2']=c
    c=0
    for j in range(0,14,2):
        r=[(t,A(t//16,j,rho_wb(t%16)),4) for t in range(64)]
        c+=cost("rd128",r)
    tot['r4']=c
    return tot


if __name__ == "__main__":
    print("row-major pitch 18 (round 5), fp64:", eval_layout(lambda r, c: r * 18 + c, 328))
    print("column-major pitch 18, D = 329, fp64:", eval_layout(lambda r, c: c * 18 + r, 329))
    print("column-major pitch 18, D = 329, fp32:", eval_layout(lambda r, c: c * 18 + r, 329, fp=32))
    print("column-major pitch 17, D = 315, fp64:", eval_layout(lambda r, c: c * 17 + r, 315))
