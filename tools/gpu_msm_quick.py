import sys, random, time, ctypes
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/oracle')
import numpy as np, pasta as P, corc as C
from halo_amd import _lib as H
H.ensure_device(0)
L=H.load()
rng=np.random.default_rng(7)
def rand_sc(n):
    a=rng.integers(0,2**63,size=(n,4),dtype=np.uint64)*2+rng.integers(0,2,size=(n,4),dtype=np.uint64)
    a[:,3]&=np.uint64(0x3fffffffffffffff); return np.ascontiguousarray(a)
for cname,cid in [('pallas',0),('vesta',1)]:
    c=P.CURVES[cname]
    g=C.srs_generate(cname, 1<<16)
    for n in [0,1,2,3,7,64,100,1000,4096,5000,1<<16]:
        sc=rand_sc(n)
        if n>5:
            sc[0]=0; sc[1]=P.int_to_limbs(P.to_mont(c.scalar-1,c.scalar)); sc[2]=sc[3]
        exp=C.msm(cname,g[:n],sc) if n else np.zeros(8,dtype=np.uint64)
        out=np.zeros(8,dtype=np.uint64)
        t=time.time(); H.check(L.halo_msm(cid,H.ptr(np.ascontiguousarray(g[:n])),n,H.ptr(sc),n,H.ptr(out))); dt=time.time()-t
        print(cname,n,np.array_equal(out,exp),'%.1f ms'%(dt*1e3))
    # all-equal scalars (skew)
    n=1<<14; sc=np.ascontiguousarray(np.repeat(rand_sc(1),n,axis=0))
    exp=C.msm(cname,g[:n],sc); out=np.zeros(8,dtype=np.uint64)
    H.check(L.halo_msm(cid,H.ptr(np.ascontiguousarray(g[:n])),n,H.ptr(sc),n,H.ptr(out)))
    print(cname,'skew',np.array_equal(out,exp))
    # srs path
    H.check(L.halo_srs_upload(cid,H.ptr(g),len(g),H.ptr(g[0]),H.ptr(g[1])))
    n=1<<15; sc=rand_sc(n); out=np.zeros(8,dtype=np.uint64)
    H.check(L.halo_msm_srs(cid,H.ptr(sc),n,H.ptr(out)))
    print(cname,'srs',np.array_equal(out,C.msm(cname,g[:n],sc)))
    # pcdl commit error
    rc=L.halo_pcdl_commit(cid,H.ptr(sc),10,10,None,H.ptr(out)); print('pcdl err',rc,H.last_error())
    # pedersen with hiding: MSM + w*S  (S = g[0] here)
    n=1000; sc=rand_sc(n); w=rand_sc(1)
    exp_pt=P.add(c, P.wrapped_to_point(c,list(C.msm(cname,g[:n],sc))), P.mul_fast(c, P.from_mont(P.limbs_to_int(w[0]),c.scalar), P.wrapped_to_point(c,list(g[0]))))
    H.check(L.halo_pedersen_commit(cid,H.ptr(w),H.ptr(np.ascontiguousarray(g[:n])),n,H.ptr(sc),n,H.ptr(out)))
    print(cname,'pedersen hiding',list(out)==P.point_to_wrapped(c,exp_pt))
    # precomputed windows
    H.check(L.halo_srs_precompute_windows(cid))
    for n in [1<<16, 1<<15, 1000, 1]:
        sc=rand_sc(n)
        H.check(L.halo_msm_srs(cid,H.ptr(sc),n,H.ptr(out)))
        print(cname,'shifted srs',n,np.array_equal(out,C.msm(cname,g[:n],sc)))
    sc=rand_sc(4096)
    H.check(L.halo_pcdl_commit(cid,H.ptr(sc),4096,4095,H.ptr(w),H.ptr(out)))
    exp_pt=P.add(c, P.wrapped_to_point(c,list(C.msm(cname,g[:4096],sc))), P.mul_fast(c, P.from_mont(P.limbs_to_int(w[0]),c.scalar), P.wrapped_to_point(c,list(g[0]))))
    print(cname,'pcdl commit hiding shifted',list(out)==P.point_to_wrapped(c,exp_pt))
