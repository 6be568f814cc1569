import sys, random
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/oracle')
import numpy as np, pasta as P, corc as C
from halo_amd import _lib as H
H.ensure_device(0)
L=H.load()
def fe_arr(vals, m): return np.array([P.int_to_limbs(P.to_mont(v,m)) for v in vals],dtype=np.uint64)
def from_arr(a, m): return [P.from_mont(P.limbs_to_int(r), m) for r in a]
ok=True
for fname,fid in [('fp',0),('fq',1)]:
    m=P.FIELDS[fname]; n=1000
    a=[random.randrange(m) for _ in range(n)]; b=[random.randrange(m) for _ in range(n)]
    a[0]=0; b[1]=0; a[2]=m-1; b[2]=m-1; a[3]=1
    A=fe_arr(a,m); B=fe_arr(b,m); out=np.zeros_like(A)
    for op,fn in [(0,lambda x,y:x*y%m),(1,lambda x,y:(x+y)%m),(2,lambda x,y:(x-y)%m),(3,lambda x,y:x*x%m),(4,lambda x,y:pow(x,-1,m) if x else 0),(5,lambda x,y:(-x)%m)]:
        H.check(L.halo_field_op(fid, op, H.ptr(A), H.ptr(B), n, H.ptr(out)))
        exp=[fn(x,y) for x,y in zip(a,b)]
        got=from_arr(out,m)
        good = got==exp and np.array_equal(out, fe_arr(exp,m))
        print(fname,'op',op,'ok' if good else 'FAIL'); ok&=good
for cname,cid in [('pallas',0),('vesta',1)]:
    c=P.CURVES[cname]; n=64
    g=C.srs_generate(cname, 200)
    A=np.ascontiguousarray(g[:n]); B=np.ascontiguousarray(g[100:100+n]); B[5]=A[5]; B[6]=0; 
    negA7=P.point_to_wrapped(c,P.neg(c,P.wrapped_to_point(c,list(A[7])))); B[7]=negA7
    out=np.zeros_like(A)
    H.check(L.halo_curve_op(cid,0,H.ptr(A),H.ptr(B),None,n,H.ptr(out)))
    exp=np.array([P.point_to_wrapped(c,P.add(c,P.wrapped_to_point(c,list(A[i])),P.wrapped_to_point(c,list(B[i])))) for i in range(n)],dtype=np.uint64)
    print(cname,'add', np.array_equal(out,exp))
    H.check(L.halo_curve_op(cid,1,H.ptr(A),None,None,n,H.ptr(out)))
    exp=np.array([P.point_to_wrapped(c,P.add(c,P.wrapped_to_point(c,list(A[i])),P.wrapped_to_point(c,list(A[i])))) for i in range(n)],dtype=np.uint64)
    print(cname,'dbl', np.array_equal(out,exp))
    ks=[random.randrange(c.scalar) for _ in range(n)]; ks[0]=0; ks[1]=1; ks[2]=c.scalar-1
    K=fe_arr(ks,c.scalar)
    H.check(L.halo_curve_op(cid,2,H.ptr(A),None,H.ptr(K),n,H.ptr(out)))
    exp=np.array([P.point_to_wrapped(c,P.mul_fast(c,ks[i],P.wrapped_to_point(c,list(A[i])))) for i in range(n)],dtype=np.uint64)
    print(cname,'smul', np.array_equal(out,exp))
