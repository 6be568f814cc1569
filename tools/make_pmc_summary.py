"""Builds profiles/pmc_summary.json from two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE; separate
passes as MI355X_MICROARCH.md prescribes).  Values are per dispatch, bytes.

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads; it is doubled for the streaming kernels (NTT passes, sort passes).  The
MSM accumulation's reads are 64-B random point gathers, for which the correction is not calibrated:
reported raw.

usage: python tools/make_pmc_summary.py <fetch_dir> <write_dir> <out.json> <source-description>
"""
import json
import sys

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from pmc_summary import load, summarise  # noqa: E402

KERNELS = {  # key -> (kernel-name substring, fetch correction)
    "msm_acc": ("k_acc<", 1.0),
    "ntt_pass": ("k_ntt_pass<halo::FpCfg, 2048, true>", 2.0),  # the 2^22 pair's full-block pass only
    "rs_scatter": ("k_rs_scatter", 2.0),
    "rs_hist": ("k_rs_hist", 2.0),
    "msm_digits": ("k_digits<", 2.0),
}


def main():
    fdir, wdir, out, src = sys.argv[1:5]
    f = summarise(load(fdir))
    w = summarise(load(wdir))
    import hashlib
    import os
    lib = os.environ.get("HALO_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "halo_amd", "lib", "libhalo_gpu.so")
    res = {
        "source": src,
        "library_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
        "units": "bytes per dispatch (FETCH_SIZE / WRITE_SIZE are KiB: x1024)",
        "correction": "gfx950 FETCH_SIZE = 1/2 of wide coalesced streaming reads: x2 for the streaming kernels; "
                      "k_acc (random 64-B point gathers) reported raw",
    }
    for key, (sub, corr) in KERNELS.items():
        fk = [k for k in f if sub in k]
        wk = [k for k in w if sub in k]
        if not fk or not wk:
            continue
        fetch = sum(f[k]["FETCH_SIZE"] * f[k]["dispatches"] for k in fk) / sum(f[k]["dispatches"] for k in fk) * 1024
        write = sum(w[k]["WRITE_SIZE"] * w[k]["dispatches"] for k in wk) / sum(w[k]["dispatches"] for k in wk) * 1024
        res[key] = {
            "kernel": fk[0].split("(")[0],
            "fetch_size_raw_bytes": fetch,
            "write_size_bytes": write,
            "fetch_correction_factor": corr,
            "hbm_bytes_per_launch": fetch * corr + write,
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
