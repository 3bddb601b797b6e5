"""Bank-conflict search over affine LDS layouts (pixel pitch PP, extra row bytes) for the
bf16x6 band kernels: LDS cycles per ds_read_b128 averaged over all (m-block, tap) reads of a
band, with the 16-lane groups of MI355X_MICROARCH.md §LDS (ideal 4).  Prints the best layouts
per geometry (ba3c_band6.h Band6<...> parameters)."""
import collections
GROUPS=[[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
GROUPS+= [[x+32 for x in g] for g in GROUPS]
def rows_rc(WS,WO,RB,pool,mb):
    out=[]
    for li in range(16):
        row=mb*16+li
        if pool:
            w=row>>2; sub=row&3; ph=w//(WO//2); pw=w%(WO//2)
            oy=2*ph+(sub>>1); ox=2*pw+(sub&1)
        else:
            oy=row//WO; ox=row%WO
        if oy>=RB: oy,ox=0,0
        out.append((oy,ox))
    return out
def cost(WS,WO,RB,KH,KW,CIN,pool,PP,RP):
    MROWS=(RB//2)*(WO//2)*4 if pool else RB*WO
    MB=(MROWS+15)//16
    tot=0;n=0
    for mb in range(MB):
        RC=rows_rc(WS,WO,RB,pool,mb)
        for kh in range(KH):
          for kw in range(KW):
            for ch in range(CIN//32):
                cyc=0
                for g in GROUPS:
                    q=collections.defaultdict(set)
                    for l in g:
                        r,x=RC[l&15]
                        a=(r+kh)*RP+(x+kw)*PP+16*(ch*4+(l>>4))
                        q[(a//16)%16].add(a)
                    cyc+=max(len(v) for v in q.values())
                tot+=cyc;n+=1
    return tot/n
geoms={'c1f':(40,36,6,5,5,32,True),'c2f':(18,14,14,5,5,32,True),'c1d':(44,40,4,5,5,32,False),'c2d':(22,18,6,5,5,64,False),
       'c1f8':(40,36,8,5,5,32,True),'c1d6':(44,40,6,5,5,32,False),'c1f4':(40,36,4,5,5,32,True)}
for name,(WS,WO,RB,KH,KW,CIN,pool) in geoms.items():
    res=[]
    for PP in range(CIN*6,CIN*6+65,16):
        for ex in range(0,16*16,16):
            RP=WS*PP+ex
            c=cost(WS,WO,RB,KH,KW,CIN,pool,PP,RP)
            res.append((round(c,3),PP,ex,round((RB+KH-1)*RP/1024,1)))
    res.sort()
    print(name,res[:5])
