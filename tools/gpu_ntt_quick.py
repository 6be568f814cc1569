import sys, random, time
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/oracle')
import numpy as np, pasta as P, corc as C
from halo_amd import _lib as H
import ctypes
H.ensure_device(0)
L=H.load()
rng=np.random.default_rng(5)
def rand_fe(n, m):
    a=rng.integers(0,2**63,size=(n,4),dtype=np.uint64)*2+rng.integers(0,2,size=(n,4),dtype=np.uint64)
    a[:,3]&=np.uint64(0x3fffffffffffffff)
    # reduce: values < 2^254 < p fine
    return np.ascontiguousarray(a)
for fname,fid in [('fp',0),('fq',1)]:
    m=P.FIELDS[fname]
    for logn in [1,2,3,5,8,10,11,12,16,17,20,22]:
        n=1<<logn
        a=rand_fe(n,m)
        exp=C.ntt(fname,a)
        got=a.copy()
        t=time.time(); H.check(L.halo_ntt(fid,H.ptr(got),logn,0)); dt=time.time()-t
        ok=np.array_equal(got,exp)
        inv=got.copy(); H.check(L.halo_ntt(fid,H.ptr(inv),logn,1))
        ok2=np.array_equal(inv,a)
        print(fname,logn,'fwd',ok,'inv',ok2, '%.1f ms'%(dt*1e3))
    # fold
    n=1<<6; a=rand_fe(3*n+5,m); out=np.zeros((n,4),dtype=np.uint64)
    H.check(L.halo_evaluate_over_domain(fid,H.ptr(a),len(a),6,H.ptr(out)))
    ai=[P.from_mont(P.limbs_to_int(r),m) for r in a]
    exp=P.ntt(ai,n,m)
    print('fold', [P.from_mont(P.limbs_to_int(r),m) for r in out]==exp)
    a=rand_fe(10,m); H.check(L.halo_evaluate_over_domain(fid,H.ptr(a),10,6,H.ptr(out)))
    ai=[P.from_mont(P.limbs_to_int(r),m) for r in a]
    print('pad', [P.from_mont(P.limbs_to_int(r),m) for r in out]==P.ntt(ai,n,m))
    co=np.zeros((n,4),dtype=np.uint64); ol=ctypes.c_size_t(0)
    H.check(L.halo_interpolate(fid,H.ptr(out),6,H.ptr(co),ctypes.byref(ol)))
    print('interp trim', ol.value==10 and np.array_equal(co[:10],a))
# device batched
import torch
x=rand_fe(4*(1<<12),P.FP_MODULUS)
d=torch.from_numpy(x.view(np.int64)).cuda()
H.check(L.halo_ntt_dev(0,ctypes.c_void_p(d.data_ptr()),12,4,0,None)); torch.cuda.synchronize()
got=d.cpu().numpy().view(np.uint64)
print('batch', all(np.array_equal(got[i<<12:(i+1)<<12], C.ntt('fp',x[i<<12:(i+1)<<12])) for i in range(4)))
