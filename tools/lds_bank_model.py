# LDS bank-conflict model of the backward sweep rounds (MI355X_MICROARCH.md LDS table):
# cycles per instruction vs conflict-free for each access pattern of riccati_knot.
# usage: python tools/lds_bank_model.py
# LDS bank-conflict model (MI355X_MICROARCH.md LDS table) for the backward sweep's rounds.
import itertools
WS, JR, QR = 24, 24, 24
def layout(NX):
    QS = 22 if NX == 14 else 13
    # BwsLds field offsets in doubles (alignas(16) for H, G, Kst, inv, dust)
    off = {}
    o = 0
    def f(name, n, al=1):
        nonlocal o
        if al > 1: o = (o + al - 1)//al*al
        off[name] = o; o += n
    f('H',196,2); f('G',14,2); f('W',7*WS); f('G2',2*WS); f('l',JR); f('ldiag',18); f('lyy2',4); f('ly2',2)
    f('U', max(JR*15 + QR*22, 3*196)); 
    off['Jt']=off['U']; off['Q']=off['U']+JR*15
    return off, QS
def cost_read64(addrs):
    # addrs: list of 64 double indices (None = inactive); 2 groups of 32; bank=(dword)%64
    cyc=0
    for g in (range(0,32),range(32,64)):
        banks={}
        for l in g:
            a=addrs[l]
            if a is None: continue
            for dw in (2*a,2*a+1):
                banks.setdefault(dw%64,set()).add(dw)
        cyc+=max([len(v) for v in banks.values()] or [0])
    return cyc  # ideal 2
def cost_write64(addrs):
    cyc=0
    for g0 in range(0,64,16):
        banks={}
        for l in range(g0,g0+16):
            a=addrs[l]
            if a is None: continue
            for dw in (2*a,2*a+1):
                banks.setdefault(dw%32,set()).add(dw)
        cyc+=max([len(v) for v in banks.values()] or [0])
    return cyc  # ideal 4
def analyse(NQ, JTS):
    NX=2*NQ; NR=NX+4
    off,QS=layout(NX); QV=QS-1
    tot={}
    # R2
    NC=NX+1; GR=64//NC; T2=(NR+GR-1)//GR
    for t in range(T2):
        rows=[ (l//NC)+GR*t for l in range(64)]
        for r in range(NQ):
            a=[off['W']+r*WS+rows[l] for l in range(64)]
            tot.setdefault('R2 W',[]).append(cost_read64(a))
        # hb read col0[b*NX] (b=coef_b(row)): j column
        a=[]
        for l in range(64):
            j=l%NC; row=rows[l]; b=row if row<NQ else row-NQ
            b=min(b,NX-1)
            a.append(off['G']+b if j==NX else off['H']+b*NX+j)
        tot.setdefault('R2 hb',[]).append(cost_read64(a))
        # write Jt
        a=[]
        for l in range(64):
            j=l%NC; g=l//NC; row=rows[l]
            if g>=GR: a.append(None); continue
            a.append(off['Q']+row*QS+QV if j==NX else off['Jt']+row*JTS+j)
        tot.setdefault('R2 wr',[]).append(cost_write64(a))
    # R3
    RG=64//NR; T3=(NR+RG-1)//RG
    for r in range(NQ):
        a=[off['Jt']+(l%NR)*JTS+NQ+r for l in range(64)]
        tot.setdefault('R3 jr',[]).append(cost_read64(a))
    for t in range(T3):
        cols=[(l//NR)+RG*t for l in range(64)]
        a=[off['Jt']+(l%NR)*JTS+(cols[l] if cols[l]<NQ else cols[l]-NQ) for l in range(64)]
        tot.setdefault('R3 jb',[]).append(cost_read64(a))
        for r in range(NQ):
            a=[off['W']+r*WS+cols[l] for l in range(64)]
            tot.setdefault('R3 W',[]).append(cost_read64(a))
        a=[None if (l//NR)>=RG else off['Q']+(l%NR)*QS+cols[l] for l in range(64)]
        tot.setdefault('R3 wr',[]).append(cost_write64(a))
    # R5
    NI=NX+1; GC=64//NI; T5=(NX+1+GC-1)//GC
    for k in range(4):
        a=[off['Q']+(NX+k)*QS+((l%NI) if (l%NI)<NX else QV) for l in range(64)]
        tot.setdefault('R5 qi',[]).append(cost_read64(a))
    for t in range(T5):
        js=[(l//NI)+GC*t for l in range(64)]
        for c in range(4):
            a=[off['Q']+(NX+c)*QS+(js[l] if js[l]<NX else QV) for l in range(64)]
            tot.setdefault('R5 qc',[]).append(cost_read64(a))
        a=[off['Q']+(l%NI)*QS+(js[l] if js[l]<NX else QV) for l in range(64)]
        tot.setdefault('R5 qij',[]).append(cost_read64(a))
        a=[off['Q']+((js[l] if js[l]<NX else 0))*QS+(l%NI) for l in range(64)]
        tot.setdefault('R5 qji',[]).append(cost_read64(a))
    for k,v in tot.items():
        ideal = 4*len(v) if 'wr' in k else 2*len(v)
        print(f"  {k:8s} instr {len(v):3d} cycles {sum(v):4d} ideal {ideal:4d}")
for NQ in (7,3):
    for JTS in (2*NQ, 2*NQ+1):
        print('NQ',NQ,'JTS',JTS); analyse(NQ,JTS)
