"""Times the device-resident naive_prover pipeline (halo_amd.prover) at n = 2^logn on one GPU."""
import json, os, sys, time
sys.path.insert(0, '/root/repo')
from halo_amd import _lib as H
from halo_amd import prover
if os.environ.get("NO_XI") == "1":  # A/B: H' = xi_0 H on the host side (halo_curve_op + H' sessions)
    del prover.DeviceBackend.ipa_many_xi
H.ensure_device(0)
for _kv in [x for x in os.environ.get('TUNE', '').split(',') if x]:  # tuning A/B: TUNE=key=value,...
    H.set_tuning(_kv.split('=')[0], int(_kv.split('=')[1]))
L = H.load()
for arg in (sys.argv[1:] or ['16', '20']):
    logn = int(arg)
    n = 1 << logn
    for curve in ('pallas',):
        cid = H.CURVES[curve]
        H.check(L.halo_srs_synthesize(cid, n, 99))
        if os.environ.get("SHIFT_C"):  # A/B: window width of the shifted SRS copies (0 = the library default)
            H.check(L.halo_srs_precompute_window_range(cid, int(os.environ["SHIFT_C"]), 0, 0))
        else:
            H.check(L.halo_srs_precompute_windows(cid))
        B = prover.DeviceBackend(curve)
        wit = prover.synthetic_witness(B, n, seed=1)
        B.sync()
        for rep in range(2):
            B.sync()
            t_ns = time.clock_gettime_ns(time.CLOCK_MONOTONIC)  # rocprofv3's trace clock (tools/prove_gaps.sh)
            out = prover.naive_prover(B, wit, n, prover.Challenges(B.m))
            print(json.dumps({"logn": logn, "curve": curve, "rep": rep, "start_ns": t_ns,
                              "times_ms": {k: round(v * 1e3, 2) for k, v in out["times"].items()}}), flush=True)
