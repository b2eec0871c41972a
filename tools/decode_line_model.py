import numpy as np, sys
sys.path.insert(0,'.')
from oracle import oracle as O
from honu_amd.workload import gen_host_batch
n=4000
hb=gen_host_batch(1,"small",0,n)
rec,off,st=O.marshal_batch(hb)
meta,info,_,_,_,tot=O.decode_batch(rec,off)
L=128
def lines(a,b):
    if b<=a: return set()
    return set(range(a//L,(b-1)//L+1))
def uvlen(x):
    k=1
    while x>=128: x>>=7; k+=1
    return k
ph={k:0 for k in ['head','w1','acl','w2','direct2','w3']}
uni=0; need=0
for i in range(n):
    beg,end=int(off[i]),int(off[i+1])
    m=meta[i]; inf=info[i]
    tstart=int(inf['data_off'])+int(inf['data_len']) if int(inf['data_len']) else beg+2
    S={}
    A=beg&~15
    S['head']=lines(A,A+16)|(lines(A+16,A+32) if (beg&15) and A+16<end else set())
    w1=tstart&~15; S['w1']=lines(w1,min(w1+256,end))
    na=int(m['acl_count']); ap=int(m['acl_off'])
    if na:
        S['acl']=set()
        for j in range(min(na,64)): S['acl']|=lines((ap+18*j)&~3,((ap+18*j)&~3)+4)
        p2=ap+18*na
    else:
        S['acl']=set(); nr=int(m['regions_count'])
        p2=(int(m['regions_off'])-uvlen(nr)) if nr else None
    if p2 is None: p2=w1+200  # rough
    w2=p2&~15; S['w2']=lines(w2,min(w2+256,end))
    sig=m['signature']; so,sl=int(sig['off']),int(sig['len'])
    if sl:
        sfr=so-uvlen(sl); p3=so+sl
        S['direct2']=lines(w2+256,sfr+uvlen(sl)) if sfr+uvlen(sl)>w2+256 else set()
    else:
        p3=max(w2+256,end-40) if end-40>w2+256 else end-40
        S['direct2']=set()
    w3=p3&~15; S['w3']=lines(w3,min(w3+256,end))
    U=set()
    for k,v in S.items(): ph[k]+=len(v)*L; U|=v
    uni+=len(U)*L
    need+= (end-tstart) + 16
print({k:round(v/n) for k,v in ph.items()}, 'sum',round(sum(ph.values())/n),'union',round(uni/n),'bytes needed',round(need/n))
# pairwise overlaps (lines fetched by two phases), including next record's head vs this record's w3
import itertools
ov={}
prevS=None
for i in range(n):
    pass
