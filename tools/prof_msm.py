import sys, time, ctypes
sys.path.insert(0,'/root/repo')
import numpy as np, torch
from halo_amd import _lib as H
H.ensure_device(0); L=H.load()
logn=int(sys.argv[1]) if len(sys.argv)>1 else 20
n=1<<logn
t=time.time(); H.check(L.halo_srs_synthesize(0,n,12345)); print('synth %.2fs'%(time.time()-t))
g=torch.Generator(device='cuda'); g.manual_seed(1)
sc=torch.randint(-2**63,2**63-1,(n,4),dtype=torch.int64,device='cuda',generator=g)
sc[:,3]&=0x0fffffffffffffff
out=np.zeros(8,dtype=np.uint64)
if len(sys.argv)>2:
    t=time.time(); H.check(L.halo_srs_precompute_windows(0)); print('precompute %.2fs'%(time.time()-t))
for i in range(3):
    torch.cuda.synchronize(); t=time.time()
    H.check(L.halo_msm_dev(0,None,ctypes.c_void_p(sc.data_ptr()),n,H.ptr(out),None))
    print('msm 2^%d: %.2f ms'%(logn,(time.time()-t)*1e3))
x=torch.randint(-2**63,2**63-1,(1<<22,4),dtype=torch.int64,device='cuda',generator=g); x[:,3]&=0x0fffffffffffffff
for i in range(3):
    torch.cuda.synchronize(); t=time.time()
    H.check(L.halo_ntt_dev(0,ctypes.c_void_p(x.data_ptr()),22,1,0,None)); torch.cuda.synchronize()
    print('ntt 2^22: %.2f ms'%((time.time()-t)*1e3))
