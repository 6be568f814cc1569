"""Times the device NTT (halo_ntt_dev, forward + inverse pair) at several sizes; checks the round trip."""
import ctypes, sys, time
sys.path.insert(0, '/root/repo')
import torch
from halo_amd import _lib as H
H.ensure_device(0)
L = H.load()
s = torch.cuda.Stream()
for kv in [a for a in sys.argv[1:] if '=' in a]:  # tuning A/B: key=value
    k, v = kv.split('=')
    H.set_tuning(k, int(v))
for logn in [int(x) for x in ([a for a in sys.argv[1:] if '=' not in a] or ['20', '22', '24'])]:
    N = 1 << logn
    g = torch.Generator(device='cuda'); g.manual_seed(logn)
    x = torch.randint(0, 2**62, (N, 4), dtype=torch.int64, device='cuda', generator=g)
    x[:, 3] &= (1 << 60) - 1
    x0 = x.clone()
    xp = ctypes.c_void_p(x.data_ptr())
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for _ in range(2):
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 0, ctypes.c_void_p(s.cuda_stream)))
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 1, ctypes.c_void_p(s.cuda_stream)))
    s.synchronize()
    ok = bool(torch.equal(x, x0))
    H.check(L.halo_profile_enable(1)); H.check(L.halo_profile_reset())
    rep = 10
    t0 = time.perf_counter()
    for _ in range(rep):
        H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 0, ctypes.c_void_p(s.cuda_stream)))
        H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 1, ctypes.c_void_p(s.cuda_stream)))
    s.synchronize()
    t1 = time.perf_counter()
    nl = ctypes.c_uint64(0); nms = ctypes.c_double(0)
    H.check(L.halo_profile_read(b"ntt_pass", ctypes.byref(nl), ctypes.byref(nms)))
    H.check(L.halo_profile_enable(0))
    ok = ok and bool(torch.equal(x, x0))
    pair = (t1 - t0) * 1e3 / rep
    print(f"logn {logn}: pair {pair:.3f} ms wall, passes {nl.value // rep} kernel-sum {nms.value / rep:.3f} ms/pair, "
          f"avg pass {nms.value / max(nl.value, 1) * 1e3:.1f} us, {N / (pair * 1e-3) / 1e9:.2f} G elem-pairs/s, roundtrip {ok}",
          flush=True)
