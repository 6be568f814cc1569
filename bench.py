#!/usr/bin/env python3
"""Benchmark of the halo proving hot path on MI355X (BASELINE.json metric: MSM points/s + NTT elems/s).

Workload at N=1 (BASELINE.json configs[1]): a 2^20-point Pippenger MSM over Pallas against the
device-resident SRS, bit-exact with the reference semantics (crates/accumulation/src/pedersen.rs:21,
pcdl::commit pcdl.rs:275).  One "step" = one MSM over a fresh batch of 2^20 scalars resident in HBM.
Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): the MSM's points are partitioned
across ranks (rank r owns SRS block r, SURVEY §8e point-partition); each rank computes its partial
sum, the partial points (64 B each) are all-gathered over RCCL and summed on the device
(halo_point_sum) -- weak scaling, value = total points of all ranks / max-over-ranks time.

Also measured (reported under "extra"): the 2^22 NTT + iNTT pair (BASELINE.json configs[2]) and, under
"extra.sizes", the 2^24 MSM (BASELINE.json configs[4] per rank) and the 2^24 NTT + iNTT pair.

The roofline object prices the dominant kernel (MSM bucket accumulation, `k_acc`): achieved =
96 B/point (64 B affine base + 32 B scalar) x points per launch / its mean launch time
from hipEvents recorded on its stream inside libhalo_gpu (halo_profile_*); traffic = the counted HBM
bytes (FETCH_SIZE / WRITE_SIZE) of this library build from profiles/pmc_summary.json.  The MSM and the
NTT are VALU-bound, so compute_roofline (k_acc) and extra.ntt.compute_roofline (k_ntt_pass) price each
kernel's counted VALU instructions class by class at the measured per-class issue rates
(profiles/issue_rates.json): frac = that issue-time ceiling / the measured launch time.
cpu_baseline times the C restatement of arkworks' msm_bigint_wnaf (oracle/oracle.c, "port") on the
host cores, rank 0, N=1.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
MSM_BYTES_PER_POINT = 96
NTT_BYTES_PER_ELEM = 64  # read + write 32 B per transform
# VALU issue ceilings per instruction class (lane-instructions/s of one MI355X, the fastest measured
# instruction of each class at 8 waves/SIMD: tools/micro/issue_bench.hip -> profiles/issue_rates.json).
# A kernel's compute ceiling is its dispatch's counted VALU instructions (rocprofv3 SQ_INSTS_VALU,
# _INT64, _INT32; profiles/pmc_summary.json "valu", stamped with the library hash) issued at these
# rates, class by class (issue costs add on a SIMD: the mixed kernels of issue_bench check it).
ISSUE_RATES_PATH = os.path.join(ROOT, "profiles", "issue_rates.json")


def valu_ceiling(valu: dict, rates: dict):
    """(issue-time ceiling in s, lane-instructions, dynamic class mix) of one dispatch.  The counted
    SQ_INSTS_VALU_INT64 splits over the 64-bit classes (mad_u64, mad_i64, ashr64, other64) and
    SQ_INSTS_VALU_INT32 over vop3 / vop2 in the proportions of the kernel's static code; the remaining
    VALU (moves, selects, lane reads) issue as VOP1 / VOP2."""
    st = valu["static_classes"]
    tot, i64, i32 = valu["valu_per_dispatch"], valu["int64_per_dispatch"], valu["int32_per_dispatch"]
    c64 = ("mad_u64", "mad_i64", "ashr64", "other64")
    s64 = max(1, sum(st[c] for c in c64))
    s32 = max(1, st["vop3"] + st["vop2"])
    n = {c: i64 * st[c] / s64 for c in c64}
    n["vop3"] = i32 * st["vop3"] / s32
    n["vop2"] = i32 * st["vop2"] / s32 + max(0.0, tot - i64 - i32)
    t = sum(n[c] * 64 / rates[c] for c in n)
    return t, tot * 64, {c: n[c] / tot for c in n}


def compute_roofline(key: str, launch_ms: float, iso_ms, pmc, lib_ok: bool, note: str):
    """The compute roofline object of one kernel (None without this build's counters / the rates)."""
    if not lib_ok or not pmc or key not in pmc or "valu" not in pmc[key] or not os.path.exists(ISSUE_RATES_PATH):
        return {"bound": "valu-issue", "frac": None, "note": "no VALU counters of this library build "
                "(tools/pmc_valu.sh) or no profiles/issue_rates.json"}
    rates = json.load(open(ISSUE_RATES_PATH))
    t_min, lanes, mix = valu_ceiling(pmc[key]["valu"], rates["rates"])
    peak = lanes / t_min
    out = {
        "bound": "valu-issue",
        "kernel": pmc[key]["valu"]["kernel"],
        "unit": "VALU lane-instructions/s",
        "achieved": lanes / (launch_ms * 1e-3) if launch_ms else None,
        "peak": peak,
        "frac": t_min / (launch_ms * 1e-3) if launch_ms else None,
        "ceiling_ms": t_min * 1e3,
        "valu_lane_instructions_per_launch": lanes,
        "dynamic_mix": mix,
        "class_rates": rates["rates"],
        "note": note + "; peak = this dispatch's counted VALU issued class by class at the measured per-class "
                       "rates (profiles/issue_rates.json, tools/micro/issue_bench.hip), so frac = ceiling time / "
                       "launch time",
    }
    if iso_ms:
        out["isolated"] = {"achieved": lanes / (iso_ms * 1e-3), "frac": t_min / (iso_ms * 1e-3),
                           "launch_ms": iso_ms}
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)  # (two streams x two scratch sets each: all four grown before timing)
    ap.add_argument("--logn", type=int, default=20, help="log2 MSM points per rank")
    ap.add_argument("--ntt-logn", type=int, default=22)
    ap.add_argument("--curve", default="pallas")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--sizes", default="24", help="extra MSM / NTT sizes (log2, comma separated) under extra.sizes")
    ap.add_argument("--dist-ntt-logn", type=int, default=24, help="distributed single NTT size (N > 1 only; 0 = off)")
    ap.add_argument("--ipa", type=int, default=1, help="measure the 2^logn IPA opening (extra.ipa_open)")
    ap.add_argument("--batch-ntt", type=int, default=1,
                    help="the prover's 42 NTT(8n) at n = 2^20 split by transform over the ranks (extra.batch_ntt)")
    ap.add_argument("--dist-ipa", type=int, default=1, help="N > 1: the sharded 2^logn opening (extra.dist_ipa)")
    ap.add_argument("--prove", type=int, default=20, help="log2 n of the naive_prover pipeline (extra.prove; 0 = off)")
    ap.add_argument("--prove-cpu", type=int, default=16, help="log2 n of the prover's CPU-baseline comparison")
    ap.add_argument("--varbase", type=int, default=1, help="variable-base MSM at 2^logn (extra.msm_varbase)")
    ap.add_argument("--commit-batch", type=int, default=1, help="16 x 2^16 batched commitments (extra.commit_batch)")
    ap.add_argument("--pcdl", default="2,4,6,8,10,12,14,16,18,20",
                    help="log2 n of the pcdl_commit / pcdl_open sweeps with w = Some (extra.pcdl; '' = off)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 over gloo (multi-rank runs on a one-GPU box)")
    ap.add_argument("--msm-streams", type=int, default=2,
                    help="streams the pipelined headline MSMs alternate over (independent MSMs; round 4, one box: "
                         "1 / 2 / 3 streams 1.26 / 1.233 / 1.296 ms/step)")
    ap.add_argument("--shift-c", type=int, default=0,
                    help="A/B: window width of the headline's shifted SRS copies (0 = the library default)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="halo_set_tuning before the run (A/B of path selections; results are identical)")
    return ap.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # HIP's default 4 hardware queues (round 4, interleaved on one box: headline 1.322 vs 1.332 ms/step,
    # opening 2^20 20.66 vs 20.73 ms, prover 2^20 199.2 vs 201.9 ms with 4 vs 8 queues)
    import torch
    import torch.distributed as dist

    from halo_amd import _lib as H
    from halo_amd.dist import allgather_points

    if args.same_device:
        local = 0
    H.ensure_device(local)
    torch.cuda.set_device(local)
    L = H.load()
    for kv in args.tune:
        k, v = kv.split("=")
        H.set_tuning(k, int(v))
    if world > 1:
        if args.same_device:  # RCCL refuses two ranks on one GPU: rehearse the protocol over gloo
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    curve = H.CURVES[args.curve]
    n = 1 << args.logn
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234 + rank)
    stream = torch.cuda.current_stream().cuda_stream
    sp = ctypes.c_void_p(stream)
    HIP = ctypes.CDLL("libamdhip64.so")
    for fn in ("hipStreamCreateWithFlags", "hipStreamDestroy", "hipEventCreateWithFlags", "hipEventRecord",
               "hipStreamWaitEvent", "hipEventDestroy"):
        getattr(HIP, fn).restype = ctypes.c_int
    HIP.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    HIP.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    HIP.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    HIP.hipEventDestroy.argtypes = [ctypes.c_void_p]
    # the headline's extra streams (--msm-streams): plain HIP streams created before the library creates
    # any of its own, so every later stream (the MSM tail streams, the IPA sessions') keeps its relative
    # placement on the 4 hardware queues (an extra stream created after them made the opening leg
    # 19.9 -> 21.2-22.1 ms)
    extra_streams = []
    for _ in range(max(1, args.msm_streams) - 1):
        hs = ctypes.c_void_p()
        if HIP.hipStreamCreateWithFlags(ctypes.byref(hs), 1) != 0:  # hipStreamNonBlocking
            raise RuntimeError("hipStreamCreateWithFlags failed")
        extra_streams.append(hs)

    def measure_msm(logn, steps, warmup, check_sync=True):
        """Pipelined MSM throughput at 2^logn points per rank against a resident synthetic SRS."""
        n = 1 << logn
        # ---- setup (outside the timed region): resident SRS = this rank's block of the global SRS
        seed = 0x48414C4F + rank  # distinct bases per rank
        H.check(L.halo_srs_synthesize(curve, n, seed))
        if args.shift_c:  # A/B of the window width of the shifted copies (every window: a full set)
            H.check(L.halo_srs_precompute_window_range(curve, args.shift_c, 0, 0))
        else:
            H.check(L.halo_srs_precompute_windows(curve))
        nbatch = max(1, min(steps, 8 if logn <= 22 else 2))
        # < 2^252 < r: valid canonical Montgomery representatives
        scalars = torch.randint(-(2**63), 2**63 - 1, (nbatch, n, 4), dtype=torch.int64, device="cuda", generator=gen)
        scalars[..., 3] &= 0x0FFFFFFFFFFFFFFF
        total_steps = warmup + steps
        d_out = torch.zeros((total_steps, 8), dtype=torch.int64, device="cuda")
        d_final = torch.zeros((total_steps, 8), dtype=torch.int64, device="cuda")
        out = np.zeros(8, dtype=np.uint64)

        torch.cuda.synchronize()  # the scalars are written before the extra streams read them
        sps = [sp] + extra_streams
        extra = extra_streams

        def run_steps(first, k):
            """k MSM steps enqueued back to back (pipelined: each step's reduction tail overlaps the
            next step's accumulation; with --msm-streams S the independent MSMs alternate over S
            streams, so a step's front can also overlap the previous step's accumulation), then the
            multi-rank combine; no host synchronisation inside."""
            for i in range(first, first + k):
                H.check(L.halo_msm_dev_async(curve, None, ctypes.c_void_p(scalars[i % nbatch].data_ptr()), n,
                                             ctypes.c_void_p(d_out[i].data_ptr()), sps[i % len(sps)]))
            for q in sps:
                H.check(L.halo_msm_join(q))
            for es in extra:  # the current stream waits for the extra streams' MSMs
                ev = ctypes.c_void_p()
                HIP.hipEventCreateWithFlags(ctypes.byref(ev), 2)  # hipEventDisableTiming
                HIP.hipEventRecord(ev, es)
                HIP.hipStreamWaitEvent(sp, ev, 0)
                HIP.hipEventDestroy(ev)
            if world > 1:
                parts = [torch.empty((k, 8), dtype=torch.int64, device="cuda") for _ in range(world)]
                dist.all_gather(parts, d_out[first:first + k].contiguous())
                stacked = torch.stack(parts, dim=1).contiguous()  # (k, world, 8)
                # the k steps' combines in one launch (a block per step; round 5 launched k lone blocks in turn)
                H.check(L.halo_point_sum_rows_dev(curve, ctypes.c_void_p(stacked.data_ptr()), k, world,
                                                  ctypes.c_void_p(d_final[first].data_ptr()), sp))

        run_steps(0, warmup)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        L.halo_profile_reset()
        L.halo_profile_enable(0 if os.environ.get("HALO_BENCH_NOPROF") == "1" else 1)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        run_steps(warmup, steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        L.halo_profile_enable(0)
        elapsed = t1 - t0
        if world > 1:
            tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        launches = ctypes.c_size_t(0)
        acc_ms = ctypes.c_double(0)
        H.check(L.halo_profile_read(b"msm_acc", ctypes.byref(launches), ctypes.byref(acc_ms)))
        acc_avg_ms = acc_ms.value / max(1, launches.value)
        # every step's result must equal the synchronous (non-pipelined) MSM of the same scalars; these
        # standalone MSMs also give k_acc's isolated launch time (the timed region's launches share the
        # GPU with the other stream's front and the previous step's tail)
        sync_ok = True
        lat = []
        L.halo_profile_reset()
        L.halo_profile_enable(0 if os.environ.get("HALO_BENCH_NOPROF") == "1" else 1)
        for i in range(min(nbatch, 4) if check_sync else 1):
            torch.cuda.synchronize()
            a0 = time.perf_counter()
            H.check(L.halo_msm_dev(curve, None, ctypes.c_void_p(scalars[i].data_ptr()), n, H.ptr(out), sp))
            lat.append((time.perf_counter() - a0) * 1e3)
            for j in range(warmup, total_steps):
                if j % nbatch == i:
                    sync_ok &= bool(np.array_equal(d_out[j].cpu().numpy().view(np.uint64), out))
        L.halo_profile_enable(0)
        H.check(L.halo_profile_read(b"msm_acc", ctypes.byref(launches), ctypes.byref(acc_ms)))
        acc_iso_ms = acc_ms.value / max(1, launches.value)
        first = d_out[0].cpu().numpy().view(np.uint64).copy() if warmup > 0 else None
        torch.cuda.synchronize()
        return elapsed, acc_avg_ms, acc_iso_ms, sync_ok, lat, scalars[0], (seed, first)

    elapsed, acc_avg_ms, acc_iso_ms, sync_ok, lat, scalars0, check0 = measure_msm(args.logn, args.steps, args.warmup)
    window_bits = L.halo_srs_window_bits(curve)

    # ---- IPA opening (pcdl::open_without_eval round loop, pcdl.rs:392-438) at 2^logn:
    # lg n rounds over the device-resident (c, z) and fold weights (weighted rounds: L/R as MSMs over
    # the resident SRS; from length 1024 on, tail rounds over the materialised G), host stand-in
    # transcript
    def measure_ipa(logn):
        n_ = 1 << logn
        R = 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001

        def fe1(v):
            m = v * (1 << 256) % R
            return np.array([(m >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)

        rng = np.random.default_rng(99)
        cs = rng.integers(0, 2**62, size=(n_, 4), dtype=np.uint64)
        hp = np.zeros(8, dtype=np.uint64)
        H.check(L.halo_srs_read(curve, 1, 1, H.ptr(hp)))
        z = fe1(12345)

        def run_open(reps=4):
            best = None
            for _ in range(reps):
                ses = ctypes.c_void_p()
                H.check(L.halo_ipa_begin(curve, H.ptr(cs), n_, H.ptr(z), H.ptr(hp), ctypes.byref(ses)))
                Lp = np.zeros(8, dtype=np.uint64)
                Rp = np.zeros(8, dtype=np.uint64)
                L.halo_profile_reset()
                L.halo_profile_enable(1)
                a0 = time.perf_counter()
                for r in range(logn):
                    H.check(L.halo_ipa_round_lr(ses, H.ptr(Lp), H.ptr(Rp)))
                    xi = (int.from_bytes(Lp.tobytes()[:16], "little") ^ (r + 1)) % R or 1
                    H.check(L.halo_ipa_fold(ses, H.ptr(fe1(xi)), H.ptr(fe1(pow(xi, -1, R)))))
                U = np.zeros(8, dtype=np.uint64)
                c0 = np.zeros(4, dtype=np.uint64)
                H.check(L.halo_ipa_end(ses, H.ptr(U), H.ptr(c0)))
                dt = (time.perf_counter() - a0) * 1e3
                L.halo_profile_enable(0)
                nl = ctypes.c_size_t(0)
                fms = ctypes.c_double(0)
                H.check(L.halo_profile_read(b"ipa_fold", ctypes.byref(nl), ctypes.byref(fms)))
                if best is None or dt < best[0]:
                    best = (dt, fms.value, U.copy())
            return best

        best = run_open()
        # the same opening with GLV folds of G every round (tuning ipa_weighted = 0): the fold kernel
        # rate for extra.cpu_ipa_fold, and the A/B of the weighted rounds; results must agree
        with H.tuning(ipa_weighted=0):
            fold_path = run_open(2)
        return {
            "workload": f"pcdl open round loop 2^{logn} (lg n rounds of L/R + fold, weighted then tail rounds), "
                        "device-resident",
            "open_ms": best[0],
            "rounds": logn,
            "glv_fold_path": {"open_ms": fold_path[0], "fold_kernels_ms": fold_path[1],
                              "same_U": bool(np.array_equal(best[2], fold_path[2]))},
        }

    ipa = measure_ipa(args.logn) if args.ipa else None

    # ---- BASELINE configs[3]: the naive_prover hot path (halo_amd.prover, protocol.rs:64-330) on the
    # device at n = 2^prove_logn, and at 2^prove_cpu_logn beside the C restatement of the same
    # pipeline on the host cores (bit-exact check of every commitment, evaluation and opening)
    def measure_prove(logn, reps=2):
        from halo_amd import prover
        n_ = 1 << logn
        H.check(L.halo_srs_synthesize(curve, n_, 0x505256 + logn))
        H.check(L.halo_srs_precompute_windows(curve))
        B = prover.DeviceBackend(args.curve)
        wit = prover.synthetic_witness(B, n_, seed=1)
        B.sync()
        best = None
        for _ in range(reps):
            out = prover.naive_prover(B, wit, n_, prover.Challenges(B.m))
            if best is None or out["times"]["total"] < best["times"]["total"]:
                best = out
        del wit
        torch.cuda.empty_cache()
        return best


    # ---- NTT + iNTT pairs (configs[2] at 2^22, and the other BASELINE sizes); rank-local, under extra
    def measure_ntt(logn, nrep=10):
        N = 1 << logn
        x = torch.randint(-(2**63), 2**63 - 1, (N, 4), dtype=torch.int64, device="cuda", generator=gen)
        x[:, 3] &= 0x0FFFFFFFFFFFFFFF
        x0 = x.clone()
        xp = ctypes.c_void_p(x.data_ptr())
        for _ in range(2):
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 0, sp))
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 1, sp))
        torch.cuda.synchronize()
        ok = bool(torch.equal(x, x0))
        # the pair's wall time without the per-pass timing events, then the passes' kernel times with them
        a0 = time.perf_counter()
        for _ in range(nrep):
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 0, sp))
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 1, sp))
        torch.cuda.synchronize()
        a1 = time.perf_counter()
        L.halo_profile_reset()
        L.halo_profile_enable(1)
        for _ in range(nrep):
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 0, sp))
            H.check(L.halo_ntt_dev(H.FP, xp, logn, 1, 1, sp))
        torch.cuda.synchronize()
        L.halo_profile_enable(0)
        nl = ctypes.c_size_t(0)
        nms = ctypes.c_double(0)
        H.check(L.halo_profile_read(b"ntt_pass", ctypes.byref(nl), ctypes.byref(nms)))
        ok = ok and bool(torch.equal(x, x0))
        pair_ms = (a1 - a0) * 1e3 / nrep
        del x, x0
        return {
            "workload": f"ntt+intt_2^{logn}_fp",
            "pair_ms": pair_ms,
            "elems_per_s_pair": N / (pair_ms * 1e-3),
            "roundtrip_bit_exact": ok,
            "passes_per_transform": int(nl.value // (2 * nrep)),
            "pass_kernel_avg_ms": nms.value / max(1, nl.value),
            "roofline_frac_pair": (2 * NTT_BYTES_PER_ELEM * N) / (pair_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        }

    # ---- evaluation algebra: pointwise product of two 2^23-element evaluation vectors
    # (the prover's 8n domain at n = 2^20), HBM-streaming: 64 B read + 32 B written per element
    def measure_evals(logn, nrep=20):
        N = 1 << logn
        a = torch.randint(-(2**63), 2**63 - 1, (N, 4), dtype=torch.int64, device="cuda", generator=gen)
        b = torch.randint(-(2**63), 2**63 - 1, (N, 4), dtype=torch.int64, device="cuda", generator=gen)
        a[:, 3] &= 0x0FFFFFFFFFFFFFFF
        b[:, 3] &= 0x0FFFFFFFFFFFFFFF
        o = torch.empty_like(a)
        res = {}
        for name, op in (("mul", 2), ("add", 0)):
            for _ in range(2):
                H.check(L.halo_evals_op_dev(H.FP, op, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                            None, 0, ctypes.c_void_p(o.data_ptr()), N, sp))
            torch.cuda.synchronize()
            a0 = time.perf_counter()
            for _ in range(nrep):
                H.check(L.halo_evals_op_dev(H.FP, op, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                            None, 0, ctypes.c_void_p(o.data_ptr()), N, sp))
            torch.cuda.synchronize()
            ms = (time.perf_counter() - a0) * 1e3 / nrep
            gbs = 96 * N / (ms * 1e-3) / 1e9
            res[name] = {"ms": ms, "achieved_GBps": gbs, "roofline_frac": gbs / HBM_PEAK_GBS}
        del a, b, o
        return {"workload": f"Evals pointwise op over 2^{logn} Fp elements (96 B/element)", **res}

    evals = measure_evals(23)

    # ---- measured HBM copy peak (reported beside the 8 TB/s spec figure): device-to-
    # device copy of 1 GiB, read + write bytes over the copy time
    def measure_copy(nbytes=1 << 30, nrep=10):
        src = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
        src.fill_(1)
        dst = torch.empty_like(src)
        for _ in range(2):
            dst.copy_(src)
        torch.cuda.synchronize()
        a0 = time.perf_counter()
        for _ in range(nrep):
            dst.copy_(src)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - a0) * 1e3 / nrep
        del src, dst
        return {"workload": "device-to-device copy of 1 GiB (torch copy kernel)", "ms": ms,
                "GBps": 2 * nbytes / (ms * 1e-3) / 1e9, "frac_of_spec": 2 * nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}

    hbm_copy = measure_copy()

    # ---- variable-base MSM (group.rs:48-50 point_dot_affine over caller bases: GLV digits, no
    # window-shifted copies), pipelined like the headline; bases = the synthetic SRS read back
    def measure_varbase(logn, steps=10, warmup=2):
        n_ = 1 << logn
        seed = 0x56424153
        H.check(L.halo_srs_synthesize(curve, n_, seed))
        bases = torch.empty((n_, 8), dtype=torch.int64, device="cuda")
        host = np.zeros((n_, 8), dtype=np.uint64)
        H.check(L.halo_srs_read(curve, 0, n_, H.ptr(host)))
        bases.copy_(torch.from_numpy(host.view(np.int64)))
        sc = torch.randint(-(2**63), 2**63 - 1, (4, n_, 4), dtype=torch.int64, device="cuda", generator=gen)
        sc[..., 3] &= 0x0FFFFFFFFFFFFFFF
        outs = torch.zeros((warmup + steps, 8), dtype=torch.int64, device="cuda")

        def run(first, k):
            for i in range(first, first + k):
                H.check(L.halo_msm_dev_async(curve, ctypes.c_void_p(bases.data_ptr()),
                                             ctypes.c_void_p(sc[i % 4].data_ptr()), n_,
                                             ctypes.c_void_p(outs[i].data_ptr()), sp))
            H.check(L.halo_msm_join(sp))

        run(0, warmup)
        torch.cuda.synchronize()
        L.halo_profile_reset()
        L.halo_profile_enable(1)
        a0 = time.perf_counter()
        run(warmup, steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - a0
        L.halo_profile_enable(0)
        nl = ctypes.c_size_t(0)
        ams = ctypes.c_double(0)
        H.check(L.halo_profile_read(b"msm_acc", ctypes.byref(nl), ctypes.byref(ams)))
        chk = (sc[0].cpu().numpy().view(np.uint64).copy(), (seed, outs[0].cpu().numpy().view(np.uint64).copy()))
        del bases, sc, outs
        return {
            "workload": f"variable-base MSM 2^{logn} over caller-supplied bases (point_dot_affine, group.rs:48-50): "
                        "GLV digits (2 x ceil(129/c) per scalar), no precomputation, pipelined",
            "points_per_s": n_ * steps / dt,
            "ms_per_msm": dt * 1e3 / steps,
            "k_acc_ms": ams.value / max(1, nl.value),
        }, chk

    varbase, varbase_chk = measure_varbase(args.logn) if args.varbase else (None, None)

    # ---- batched commitments (halo_msm_batch_dev; protocol.rs:114,263: 16 commits per round)
    def measure_commit_batch(logn, k=16, reps=5):
        n_ = 1 << logn
        H.check(L.halo_srs_synthesize(curve, n_, 0x42415443))
        H.check(L.halo_srs_precompute_windows(curve))
        sc = torch.randint(-(2**63), 2**63 - 1, (k, n_, 4), dtype=torch.int64, device="cuda", generator=gen)
        sc[..., 3] &= 0x0FFFFFFFFFFFFFFF
        ptrs = (ctypes.c_void_p * k)(*[sc[i].data_ptr() for i in range(k)])
        lens = (ctypes.c_size_t * k)(*([n_] * k))
        out = torch.zeros((k, 8), dtype=torch.int64, device="cuda")
        out_ref = torch.zeros((k, 8), dtype=torch.int64, device="cuda")
        for i in range(k):  # per-MSM pipelined path, for the equality check
            H.check(L.halo_msm_dev_async(curve, None, ctypes.c_void_p(sc[i].data_ptr()), n_,
                                         ctypes.c_void_p(out_ref[i].data_ptr()), sp))
        H.check(L.halo_msm_join(sp))
        H.check(L.halo_msm_batch_dev(curve, ptrs, lens, k, ctypes.c_void_p(out.data_ptr()), sp))
        H.check(L.halo_msm_join(sp))
        torch.cuda.synchronize()
        a0 = time.perf_counter()
        for _ in range(reps):
            H.check(L.halo_msm_batch_dev(curve, ptrs, lens, k, ctypes.c_void_p(out.data_ptr()), sp))
            H.check(L.halo_msm_join(sp))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - a0) * 1e3 / reps
        same = bool(torch.equal(out, out_ref))
        del sc
        return {"workload": f"{k} commitments of 2^{logn} coefficients in one halo_msm_batch_dev call "
                            "(one MSM, (polynomial, bucket) keys)", "ms_per_batch": ms,
                "points_per_s": k * n_ / (ms * 1e-3), "equals_per_msm_path": same}

    commit_batch = measure_commit_batch(16) if args.commit_batch else None

    # ---- the reference's own criterion shapes (crates/accumulation/benches/pcdl.rs:35-79): pcdl_commit
    # and pcdl_open with w = Some over n = 2^2..2^20, Pallas; host buffers in and out as the Rust API
    # has them; the open includes v = p(z), the hiding branch and the lg n rounds with a stand-in
    # transcript (SHA-256; the Poseidon sponge is host logic, ~us per absorb)
    def measure_pcdl(lgs):
        from halo_amd import pcdl as P_
        top = max(lgs)
        N = 1 << top
        H.check(L.halo_srs_synthesize(curve, N, 0x50434C44))
        G = np.zeros((N, 8), dtype=np.uint64)
        H.check(L.halo_srs_read(curve, 0, N, H.ptr(G)))
        H.check(L.halo_srs_upload(curve, H.ptr(G), N, H.ptr(G[0]), H.ptr(G[1])))  # S = G_0, H = G_1 (synthetic)
        H.check(L.halo_srs_precompute_windows(curve))
        rng = np.random.default_rng(3)

        def fes(k):
            a = rng.integers(0, 2**63, size=(k, 4), dtype=np.uint64)
            a[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
            return np.ascontiguousarray(a)

        res = {}
        inputs = {}
        for lg in lgs:
            n_ = 1 << lg
            p_, w_, z_ = fes(n_), fes(1)[0], fes(1)[0]
            q_, wb_ = fes(n_ - 1), fes(1)[0]
            C = P_.commit(p_, n_ - 1, w_, args.curve)
            reps = 10 if lg <= 14 else 3
            a0 = time.perf_counter()
            for _ in range(reps):
                C = P_.commit(p_, n_ - 1, w_, args.curve)
            t_commit = (time.perf_counter() - a0) / reps
            P_.open(p_, C, n_ - 1, z_, w=w_, transcript=P_.StandInTranscript(args.curve), q=q_, w_bar=wb_,
                    curve=args.curve)
            reps = 5 if lg <= 14 else 2
            a0 = time.perf_counter()
            for _ in range(reps):
                pi = P_.open(p_, C, n_ - 1, z_, w=w_, transcript=P_.StandInTranscript(args.curve), q=q_, w_bar=wb_,
                             curve=args.curve)
            t_open = (time.perf_counter() - a0) / reps
            res[f"2^{lg}"] = {"commit_ms": t_commit * 1e3, "open_ms": t_open * 1e3}
            inputs[lg] = (p_, w_, z_, q_, wb_, C, pi)
        return res, inputs, G  # G: the sweep's SRS (S = G_0, H = G_1), kept for the CPU leg

    pcdl_lgs = [int(v) for v in args.pcdl.split(",") if v.strip()] if world == 1 else []
    pcdl_sweep, pcdl_inputs, pcdl_sh = measure_pcdl(pcdl_lgs) if pcdl_lgs else (None, None, None)

    # ---- BASELINE configs[4] as named: one 2^lg-point MSM window-partitioned across the ranks
    # (halo_amd.dist.window_range): every rank the same SRS and scalars (broadcast from rank 0 over
    # RCCL), rank r the windows of its range, partials all-gathered + summed on the device
    def measure_window_partition(lg, reps=4):
        from halo_amd.dist import partition_window_bits, window_range
        n_ = 1 << lg
        H.check(L.halo_srs_synthesize(curve, n_, 0x57494E44))  # same seed on every rank
        # a window width whose W divides the world (16 windows of 16 bits over 8 ranks), and on each
        # rank only the copies of its own windows (2 x 2^24 x 64 B instead of all 15 or 16)
        c = partition_window_bits(world)
        W = -(-255 // c)
        lo, hi = window_range(W, rank, world)
        H.check(L.halo_srs_precompute_window_range(curve, c, lo, hi))
        sc = torch.empty((n_, 4), dtype=torch.int64, device="cuda")
        if rank == 0:
            sc.copy_(torch.randint(-(2**63), 2**63 - 1, (n_, 4), dtype=torch.int64, device="cuda", generator=gen))
            sc[:, 3] &= 0x0FFFFFFFFFFFFFFF
        part = torch.zeros((1, 8), dtype=torch.int64, device="cuda")
        parts = [torch.empty_like(part) for _ in range(world)]
        res = torch.zeros(8, dtype=torch.int64, device="cuda")

        def one(bcast):
            if bcast:
                dist.broadcast(sc, 0)
            H.check(L.halo_msm_srs_windows_dev(curve, ctypes.c_void_p(sc.data_ptr()), n_, lo, hi,
                                               ctypes.c_void_p(part.data_ptr()), sp))
            H.check(L.halo_msm_join(sp))
            dist.all_gather(parts, part)
            st = torch.cat(parts).contiguous()
            H.check(L.halo_point_sum_dev(curve, ctypes.c_void_p(st.data_ptr()), world, 64,
                                         ctypes.c_void_p(res.data_ptr()), sp))

        out = {}
        for bcast in (True, False):
            one(True)
            torch.cuda.synchronize()
            dist.barrier()
            a0 = time.perf_counter()
            for _ in range(reps):
                one(bcast)
            torch.cuda.synchronize()
            dist.barrier()
            tt = torch.tensor([time.perf_counter() - a0], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            out["ms_per_msm_with_broadcast" if bcast else "ms_per_msm_resident_scalars"] = float(tt.item()) * 1e3 / reps
        # the collective alone: the scalar broadcast (n x 32 B from rank 0) with no MSM behind it
        dist.broadcast(sc, 0)
        torch.cuda.synchronize()
        dist.barrier()
        a0 = time.perf_counter()
        for _ in range(reps):
            dist.broadcast(sc, 0)
        torch.cuda.synchronize()
        dist.barrier()
        tt = torch.tensor([time.perf_counter() - a0], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        out["ms_broadcast_only"] = float(tt.item()) * 1e3 / reps
        out["broadcast_GB_per_s"] = n_ * 32 / (out["ms_broadcast_only"] * 1e-3) / 1e9
        # the partitioned result must equal rank 0's whole MSM of the same scalars
        ok = None
        if rank == 0:
            whole = torch.zeros(8, dtype=torch.int64, device="cuda")
            H.check(L.halo_msm_dev_async(curve, None, ctypes.c_void_p(sc.data_ptr()), n_,
                                         ctypes.c_void_p(whole.data_ptr()), sp))
            H.check(L.halo_msm_join(sp))
            torch.cuda.synchronize()
            ok = bool(torch.equal(whole, res))
        del sc
        return {"workload": f"one 2^{lg}-point MSM, {W} windows of {c} bits split over {world} ranks (window_range; "
                            f"each rank holds only its own windows' shifted copies), scalars broadcast from rank 0, "
                            f"partials all-gathered", "windows_of_rank0": [lo, hi],
                "points_per_s_with_broadcast": n_ / (out["ms_per_msm_with_broadcast"] * 1e-3),
                "points_per_s_resident_scalars": n_ / (out["ms_per_msm_resident_scalars"] * 1e-3),
                "matches_single_gpu": ok, "scaling": "strong", **out}

    ntt_main = measure_ntt(args.ntt_logn)
    ntt_main["workload"] += " (BASELINE.json configs[2])"
    sizes = {}
    ntt24_keys = []
    size_checks = {}  # 2^lg MSM: (scalars[0] on the host, SRS seed, result), verified in the CPU leg
    for lg in [int(v) for v in args.sizes.split(",") if v.strip()]:
        # 8 pipelined MSMs after 4 warm-up ones (round 5 timed 4 after 2: the two scratch sets of each
        # stream's slot not yet grown to this size were allocated inside the timed region, ~9 GB each at
        # 2^24, and the last MSM's exposed tail was a quarter of the region)
        ksz = 8
        e, a_ms, _, ok, lt, sc0, chk = measure_msm(lg, ksz, 4, check_sync=False)
        if world == 1 and not args.no_cpu:
            size_checks[lg] = (sc0.cpu().numpy().view(np.uint64).copy(), chk)
        del sc0
        sizes[f"msm_2^{lg}"] = {
            "points_per_s": (1 << lg) * world * ksz / e,
            "ms_per_msm": e * 1e3 / ksz,
            "steps": ksz,
            "k_acc_ms": a_ms,
            "single_latency_ms": lt[0] if lt else None,
            "roofline_frac": MSM_BYTES_PER_POINT * (1 << lg) * world * ksz / e / 1e9 / HBM_PEAK_GBS,
        }
        sizes[f"ntt_2^{lg}"] = measure_ntt(lg, nrep=4)
        if lg == 24:  # the 8-bit passes' kernel, priced like the 2^22 pair's (after the PMC load below)
            ntt24_keys.append(f"ntt_2^{lg}")
        torch.cuda.empty_cache()
        if world > 1 and (world & (world - 1)) == 0:
            # BASELINE configs[4]: one 2^lg-point MSM partitioned across the ranks (strong scaling)
            lr = lg - (world.bit_length() - 1)
            e, a_ms, _, ok, lt, _, _ = measure_msm(lr, 4, 2, check_sync=False)
            sizes[f"msm_2^{lg}_partitioned"] = {
                "points_per_s": (1 << lg) * 4 / e,
                "ms_per_msm": e * 1e3 / 4,
                "points_per_rank": 1 << lr,
                "scaling": "strong",
            }
            torch.cuda.empty_cache()
            sizes[f"msm_2^{lg}_window_partitioned"] = measure_window_partition(lg)
            torch.cuda.empty_cache()

    # ---- distributed single NTT (four-step, RCCL all-to-all; halo_amd.dist.sharded_ntt), N > 1 only
    dist_ntt = None
    if world > 1 and args.dist_ntt_logn:
        from halo_amd.dist import GpuNttOps, sharded_ntt, torch_alltoall
        lg = args.dist_ntt_logn
        per = (1 << lg) // world
        xl = torch.randint(-(2**63), 2**63 - 1, (per, 4), dtype=torch.int64, device="cuda", generator=gen)
        xl[:, 3] &= 0x0FFFFFFFFFFFFFFF
        ops = GpuNttOps(H.FP)
        a2a = torch_alltoall(dist)
        y = sharded_ntt(xl, lg, False, ops, rank, world, a2a)
        z = sharded_ntt(y, lg, True, ops, rank, world, a2a)
        torch.cuda.synchronize()
        ok = torch.tensor([int(torch.equal(z, xl))], device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        reps = 5
        dist.barrier()
        torch.cuda.synchronize()
        a0 = time.perf_counter()
        for _ in range(reps):
            y = sharded_ntt(xl, lg, False, ops, rank, world, a2a)
            z = sharded_ntt(y, lg, True, ops, rank, world, a2a)
        torch.cuda.synchronize()
        dist.barrier()
        tt = torch.tensor([time.perf_counter() - a0], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        pair_ms = float(tt.item()) * 1e3 / reps
        dist_ntt = {
            "workload": f"distributed ntt+intt_2^{lg}_fp over {world} ranks (four-step, 3 RCCL all-to-alls each way)",
            "pair_ms": pair_ms,
            "elems_per_s_pair": (1 << lg) / (pair_ms * 1e-3),
            "roundtrip_bit_exact": bool(ok.item()),
        }
        del xl, y, z

    # ---- the prover's NTTs sharded by transform: round 0 of the 2^20
    # naive_prover evaluates 42 polynomials of degree < 2^20 over the 8n = 2^23 domain (protocol.rs:88-106),
    # independent transforms, so rank r takes transforms r, r + P, ... with no exchange at all
    # (halo_ntt_dev_zero_tail, one batched call per rank).  Strong scaling over the fixed 42 transforms;
    # measured at every N (N = 1: all 42 on one GPU), beside the four-step dist_ntt
    def measure_batch_ntt(lg=23, lg_nz=20, T=42, reps=3):
        N_ = 1 << lg
        mine = [t for t in range(T) if t % world == rank]
        x0 = torch.zeros((len(mine), N_, 4), dtype=torch.int64, device="cuda")
        for i, t in enumerate(mine):  # transform t's coefficients depend on t only (any rank can recompute it)
            gt = torch.Generator(device="cuda")
            gt.manual_seed(7000 + t)
            x0[i, :1 << lg_nz] = torch.randint(-(2**63), 2**63 - 1, (1 << lg_nz, 4), dtype=torch.int64, device="cuda",
                                               generator=gt)
        x0[:, :, 3] &= 0x0FFFFFFFFFFFFFFF
        x = torch.empty_like(x0)
        xp = ctypes.c_void_p(x.data_ptr())
        best = None
        for rep in range(reps + 1):  # (the first call builds the twiddle tables: untimed)
            x.copy_(x0)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            a0 = time.perf_counter()
            if mine:
                H.check(L.halo_ntt_dev_zero_tail(H.FP, xp, lg, len(mine), 1 << lg_nz, sp))
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            dt = time.perf_counter() - a0
            if world > 1:
                tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                dt = float(tt.item())
            if rep and (best is None or dt < best):
                best = dt
        wts = (torch.arange(N_ * 4, device="cuda", dtype=torch.int64) % 1009 + 1).view(N_, 4)

        def digest(y):  # per transform: an integer weighted sum (exact, order-free mod 2^64)
            return torch.stack([(y[i] * wts).sum() for i in range(y.shape[0])])

        dig = torch.zeros(T, dtype=torch.int64, device="cuda")
        if mine:
            dig[mine] = digest(x)
        # round trip: the inverse transforms give back the coefficients (and the zero tail)
        if mine:
            H.check(L.halo_ntt_dev(H.FP, xp, lg, len(mine), 1, sp))
        torch.cuda.synchronize()
        ok = torch.tensor([int(torch.equal(x, x0))], device="cuda")
        matches = None
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            dist.all_reduce(dig, op=dist.ReduceOp.SUM)  # each transform's digest from its owner (others add 0)
            if rank == 0:  # rank 0 recomputes every transform alone (the one-GPU result)
                y = torch.zeros((1, N_, 4), dtype=torch.int64, device="cuda")
                one = []
                for t in range(T):
                    gt = torch.Generator(device="cuda")
                    gt.manual_seed(7000 + t)
                    y.zero_()
                    y[0, :1 << lg_nz] = torch.randint(-(2**63), 2**63 - 1, (1 << lg_nz, 4), dtype=torch.int64,
                                                      device="cuda", generator=gt)
                    y[0, :, 3] &= 0x0FFFFFFFFFFFFFFF
                    H.check(L.halo_ntt_dev_zero_tail(H.FP, ctypes.c_void_p(y.data_ptr()), lg, 1, 1 << lg_nz, sp))
                    one.append(digest(y)[0])
                matches = bool(torch.equal(torch.stack(one), dig))
                del y
        del x, x0, wts
        torch.cuda.empty_cache()
        return {"workload": f"naive_prover round 0's {T} NTT(8n) at n = 2^{lg_nz} (zero-tail 2^{lg} transforms of "
                            f"degree < 2^{lg_nz} polynomials, halo_ntt_dev_zero_tail) split by transform over {world} "
                            f"rank(s), no exchange", "ms": best * 1e3, "transforms_per_s": T / best,
                "transforms_on_rank0": len([t for t in range(T) if t % world == 0]), "scaling": "strong",
                "roundtrip_bit_exact": bool(ok.item()), "matches_single_gpu": matches}

    batch_ntt = measure_batch_ntt() if args.batch_ntt else None

    # ---- distributed IPA opening (strided shards, halo_amd.dist.sharded_ipa_rounds), N > 1 only:
    # every rank synthesizes the same 2^logn SRS and then keeps only its shard G[i P + r] resident (with
    # its window-shifted copies), so each shard runs the weighted rounds (GpuWeightedIpaOps); the
    # per-round L_r, R_r are all-gathered on the device and summed there (torch_reduce_lr)
    dist_ipa = None
    if world > 1 and args.ipa and args.dist_ipa:
        from halo_amd import pcdl as PC
        from halo_amd.dist import (GpuWeightedIpaOps, sharded_ipa_rounds, torch_gather_arrays, torch_reduce_lr,
                                   torch_reduce_lr_dev)
        from halo_amd.group import PublicParams
        n_ = 1 << args.logn
        H.check(L.halo_srs_synthesize(curve, n_, 777))
        G = np.zeros((n_, 8), dtype=np.uint64)
        H.check(L.halo_srs_read(curve, 0, n_, H.ptr(G)))
        Rm = 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001

        def fe1(v):
            m = v * (1 << 256) % Rm
            return np.array([(m >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)

        rng = np.random.default_rng(99)
        cs = rng.integers(0, 2**62, size=(n_, 4), dtype=np.uint64)
        z_ark = fe1(12345)
        hp = G[1].copy()
        ks = {"k": 0}

        def challenge(xi_prev, Lp, Rp):
            ks["k"] += 1
            return fe1((int.from_bytes(Lp.tobytes()[:16], "little") ^ ks["k"]) % Rm or 1)

        def inverse(x):
            v = int.from_bytes(x.tobytes(), "little") * pow(1 << 256, -1, Rm) % Rm
            return fe1(pow(v, -1, Rm))

        ref = None
        if rank == 0:  # the unsharded opening of the same instance on one GPU (weighted rounds)
            H.check(L.halo_srs_precompute_windows(curve))
            ref = PC.ipa_rounds(cs, z_ark, hp, challenge, inverse, args.curve)
        PublicParams.upload(args.curve, np.ascontiguousarray(G[rank::world]), precompute_windows=True)
        shard = (np.ascontiguousarray(cs[rank::world]), z_ark)
        ops = GpuWeightedIpaOps(args.curve, rank, world)
        gather = torch_gather_arrays(dist, "cuda")

        def run_sharded(device_lr):
            reduce_lr = (torch_reduce_lr_dev if device_lr else torch_reduce_lr)(dist, args.curve, "cuda")
            best, res = None, None
            for _ in range(3):
                ks["k"] = 0
                dist.barrier()
                torch.cuda.synchronize()
                a0 = time.perf_counter()
                res = sharded_ipa_rounds([shard], hp, challenge, inverse, ops, world, gather, reduce_lr,
                                         device_lr=device_lr)
                torch.cuda.synchronize()
                tt = torch.tensor([time.perf_counter() - a0], dtype=torch.float64, device="cuda")
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                best = float(tt.item()) if best is None else min(best, float(tt.item()))
            same = None
            if rank == 0:
                Ls, Rs, U, c0 = res
                Ls1, Rs1, U1, c1 = ref
                same = all(np.array_equal(a_, b_) for a_, b_ in zip(Ls + Rs + [U, c0], Ls1 + Rs1 + [U1, c1]))
            return best, same

        best_dev, same_dev = run_sharded(True)
        best_host, same_host = run_sharded(False)
        dist_ipa = {
            "workload": f"pcdl open 2^{args.logn} sharded over {world} ranks (rank r: resident SRS shard G[r::P] "
                        f"with window-shifted copies, weighted rounds; per round the ranks' L_r, R_r stay on the "
                        f"device (halo_ipa_round_lr_dev), one RCCL all-gather, an XYZZ sum on the device and one "
                        f"D2H for the transcript; last lg P rounds collapsed)",
            "open_ms": best_dev * 1e3,
            "matches_single_gpu": same_dev,
            "host_pair_reduce": {"open_ms": best_host * 1e3, "matches_single_gpu": same_host,
                                 "note": "round 5's reduce: each rank's pair through the host (D2H, affine, H2D) "
                                         "before the gather, affine device sums"},
        }
        del G, cs

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    total_points = n * world * args.steps
    value = total_points / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    acc_bytes = MSM_BYTES_PER_POINT * n
    achieved = acc_bytes / (acc_avg_ms * 1e-3) / 1e9 if acc_avg_ms > 0 else 0.0

    # PMC traffic of k_acc from the committed counter passes, used only when they were measured on
    # this very library build (library_sha256 stamp); otherwise null with the reason
    traffic = None
    traffic_note = "no profiles/pmc_summary.json"
    pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    pmc, pmc_ok = None, False
    if os.path.exists(pmc_path):
        try:
            import hashlib
            pmc = json.load(open(pmc_path))
            lib_sha = hashlib.sha256(open(H.LIB_PATH, "rb").read()).hexdigest()
            pmc_ok = pmc.get("library_sha256") == lib_sha
            if pmc_ok:
                traffic = pmc.get("msm_acc", {}).get("hbm_bytes_per_launch")
                traffic_note = "rocprofv3 FETCH_SIZE + WRITE_SIZE (separate passes) of this library build, " \
                               "profiles/pmc_summary.json"
            else:
                traffic_note = "profiles/pmc_summary.json was measured on another library build: not used"
        except (OSError, ValueError):
            traffic = None

    cpu = None
    cpu_ntt = cpu_fold = None
    verified = {}
    if not args.no_cpu and world == 1:
        cpu = cpu_baseline(L, H, curve, n, scalars0, out_check=True, budget_s=args.cpu_seconds)
        cpu_ntt = cpu_ntt_baseline(L, H, args.ntt_logn, sp, ntt_main)
        cpu_fold = cpu_fold_baseline(L, H, curve, 13, ipa)
        # known-log identity checks of the measured MSMs (oracle dot product + generator multiple)
        verified["msm_2^%d" % args.logn] = cpu_known_log_check(args.curve, scalars0.cpu().numpy().view(np.uint64),
                                                               check0)
        for lg, (sc_h, chk) in size_checks.items():
            sizes[f"msm_2^{lg}"]["verified"] = cpu_known_log_check(args.curve, sc_h, chk)
        if varbase_chk is not None:
            varbase["verified"] = cpu_known_log_check(args.curve, varbase_chk[0], varbase_chk[1])
        if pcdl_sweep:
            cpu_pcdl_baseline(args.curve, pcdl_sweep, pcdl_inputs, pcdl_sh, L, H, curve)

    # after the MSM CPU leg (which reads the MSM's resident SRS back)
    prove = None
    if args.prove and world == 1:
        main_out = measure_prove(args.prove)
        prove = {
            "workload": f"naive_prover hot path at n = 2^{args.prove} (BASELINE.json configs[3]): 17 iNTT(n) + "
                        f"42 NTT(8n), 33 commits, 14 + 3 FFT products, gate constraints over 8n, quotient, "
                        f"3 IPA openings, 91 evaluations; synthetic witness, stand-in transcript",
            "n": 1 << args.prove,
            "ms": {k: v * 1e3 for k, v in main_out["times"].items()},
        }
        # the prover's kernels against their VALU-issue ceilings (tools/pmc_prove.sh: kernel statistics and
        # VALU counters of the same 2^20 prove, stamped with the library hash; attached only for this build)
        pv_path = os.path.join(ROOT, "profiles", "prove_valu.json")
        if args.prove == 20 and os.path.exists(pv_path):
            import hashlib
            pv = json.load(open(pv_path))
            if pv.get("library_sha256") == hashlib.sha256(open(H.LIB_PATH, "rb").read()).hexdigest():
                prove["kernel_rooflines"] = {
                    "source": "profiles/prove_valu.json (" + pv["source"] + ")",
                    "kernels": {k: {f: e.get(f) for f in ("calls", "mean_us", "share", "ceiling_us", "compute_frac")}
                                for k, e in pv["kernels"].items()}}
            else:
                prove["kernel_rooflines"] = {"note": "profiles/prove_valu.json was measured on another library build"}
        if not args.no_cpu:
            prove["verified"] = cpu_prove_check(L, H, curve, args.curve, 1 << args.prove, main_out)
        if not args.no_cpu and args.prove_cpu:
            small = measure_prove(args.prove_cpu)
            prove["at_cpu_size"] = {"n": 1 << args.prove_cpu, "gpu_ms": {k: v * 1e3 for k, v in small["times"].items()}}
            prove["cpu"] = cpu_prove_baseline(L, H, curve, args.curve, args.prove_cpu, small)

    madds = n * (-(-255 // window_bits)) if window_bits else 0  # one mixed addition per nonzero digit
    # the counted VALU of k_acc applies to the configuration it was counted on (2^20 points, 17-bit windows)
    headline_shape = args.logn == 20 and window_bits == 17
    acc_compute = compute_roofline("msm_acc", acc_avg_ms, acc_iso_ms, pmc, pmc_ok and headline_shape,
                                   "k_acc over the timed region's mean launch time (live, beside the other stream's "
                                   "front); isolated: the standalone MSMs after it")
    acc_compute["modmul_rate"] = {
        "achieved": madds * 10 / (acc_avg_ms * 1e-3) if acc_avg_ms > 0 else None,
        "unit": "modmul/s", "note": "XYZZ mixed additions (8M + 2S, counted as 10) per launch over the live launch "
                                    "time (informational: not a ceiling)"}
    for key in ntt24_keys:
        sizes[key]["compute_roofline"] = compute_roofline(
            "ntt_pass_1024", sizes[key].get("pass_kernel_avg_ms"), None, pmc, pmc_ok,
            "k_ntt_pass<Fp, 1024, full blocks> (the 8-bit Stockham pass, 6 per 2^24 pair) over its mean launch time")
    if ntt_main is not None:
        ntt_main["compute_roofline"] = compute_roofline(
            "ntt_pass", ntt_main.get("pass_kernel_avg_ms"), None, pmc, pmc_ok and args.ntt_logn == 22,
            "k_ntt_pass<Fp, 2048, full blocks> (the 11-bit Stockham pass, 4 per pair) over its mean launch time in the pair loop")

    line = {
        "metric": "MSM points/sec (Pippenger, Pallas, 2^20 points, resident SRS)",
        "value": value,
        "unit": "points/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 limbs (255-bit Montgomery field, integer)",
        "data": "synthetic: uniform random scalars; SRS bases G_j = k_j*(-1,2) with seeded k_j (known discrete logs)",
        "config": {
            "workload": f"msm_2^{args.logn}_pallas_resident_srs (BASELINE.json configs[1]; point-partitioned across ranks)",
            "points_per_rank": n,
            "window_bits": window_bits,
            "parallelism": f"point-partition x{world}, RCCL all-gather of partial sums",
            "world_size_reported": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "pipelining": f"steps enqueued back to back over {max(1, args.msm_streams)} stream(s): step k's reduction "
                          "tail overlaps step k+1's accumulation, and with two streams step k+1's front also "
                          "overlaps step k's accumulation",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_acc (MSM bucket accumulation)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_note": traffic_note,
            "algorithmic_bytes_per_launch": acc_bytes,
            "avg_launch_ms": acc_avg_ms,
            "isolated_launch_ms": acc_iso_ms,
            "note": "the MSM is bound by 255-bit modular multiplication on the VALU, not HBM (SURVEY §7 hard part 1); "
                    "avg_launch_ms is over the timed region's launches, which share the GPU with the other stream's "
                    "front and the previous step's tail, isolated_launch_ms over the standalone MSMs after it",
        },
        "cpu_baseline": cpu,
        "compute_roofline": acc_compute,
        "extra": {
            "msm_single_latency_ms": min(lat) if lat else None,
            "pipelined_equals_sync": sync_ok,
            "ntt": ntt_main,
            "sizes": sizes,
            "dist_ntt": dist_ntt,
            "dist_ipa": dist_ipa,
            "batch_ntt": batch_ntt,
            "ipa_open": ipa,
            "evals_op": evals,
            "hbm_copy": hbm_copy,
            "cpu_ntt": cpu_ntt,
            "prove": prove,
            "cpu_ipa_fold": cpu_fold,
            "msm_varbase": varbase,
            "commit_batch": commit_batch,
            "pcdl": pcdl_sweep,
            "verified": verified,
        },
    }
    print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(L, H, curve, n, scalars_dev, out_check, budget_s):
    """Rank 0, N=1 only: the C port of arkworks msm_bigint_wnaf (oracle/oracle.c) on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import corc  # noqa: E402  (oracle: only the cpu_baseline leg may load it)

    bases = np.zeros((n, 8), dtype=np.uint64)
    H.check(L.halo_srs_read(curve, 0, n, H.ptr(bases)))
    sc = np.ascontiguousarray(scalars_dev.cpu().numpy().view(np.uint64))
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = min(threads, 16)
    gpu_out = np.zeros(8, dtype=np.uint64)
    H.check(L.halo_msm(curve, H.ptr(bases), n, H.ptr(sc), n, H.ptr(gpu_out)))
    reps = 0
    t0 = time.perf_counter()
    cpu_out = None
    while True:
        cpu_out = corc.msm("pallas" if curve == 0 else "vesta", bases, sc, threads=threads)
        reps += 1
        if time.perf_counter() - t0 >= budget_s or reps >= 5:
            break
    dt = (time.perf_counter() - t0) / reps
    # the same restatement on one thread, over a 2^16-point prefix of the same inputs
    n1 = min(n, 1 << 16)
    t1 = time.perf_counter()
    corc.msm("pallas" if curve == 0 else "vesta", np.ascontiguousarray(bases[:n1]), np.ascontiguousarray(sc[:n1]),
             threads=1)
    one_thread = n1 / (time.perf_counter() - t1)
    return {
        "value": n / dt,
        "unit": "points/s",
        "cores": threads,
        "single_thread": {"value": one_thread, "unit": "points/s", "sample": f"1 x 2^{n1.bit_length() - 1}-point "
                          "prefix of the same MSM, 1 thread"},
        "kind": "port",
        "sample": f"{reps} x full 2^{n.bit_length() - 1}-point MSM (same bases/scalars as the GPU), C restatement of "
                  f"ark-ec 0.5 msm_bigint_wnaf, c={corc.msm_window_size(n)}, OpenMP over windows",
        "gpu_matches_cpu": bool(np.array_equal(cpu_out, gpu_out)) if out_check else None,
    }


def cpu_known_log_check(cname, scalars_host, chk):
    """The MSM result against (sum_j s_j k_j) G, k_j the synthetic SRS's discrete logs (oracle)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import corc  # noqa: E402  (oracle: the checker, CPU leg only)
    seed, got = chk
    if got is None:
        return None
    n = len(scalars_host)
    k = corc.synth_scalars(seed, n)
    return bool(np.array_equal(corc.known_log_msm(cname, np.ascontiguousarray(scalars_host), k), got))


def cpu_prove_check(L, H, curve, cname, n, out):
    """The three openings of the measured prove pass the oracle's succinct_check (pcdl.rs:483-554,
    with the prover's challenges) and the decider U == commit(h) (pcdl.rs:579-581, oracle MSM)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import corc  # noqa: E402
    import pcdl_check  # noqa: E402
    srs = np.zeros((n, 8), dtype=np.uint64)
    H.check(L.halo_srs_read(curve, 0, n, H.ptr(srs)))
    res = {}
    for key in ("q_r", "q_r_omega", "acc"):
        q = out[key]
        try:
            pcdl_check.succinct_check(cname, q["C"], n - 1, q["z"], q["v"], q["Ls"], q["Rs"], q["U"], q["c"], q["xis"],
                                      srs[1])
            ok = True
        except AssertionError:
            ok = False
        res[key] = ok and pcdl_check.decider_commit_matches(cname, q["U"], q["xis"], srs, corc.msm)
    return res


def cpu_pcdl_baseline(cname, sweep, inputs, G, L, H, curve):
    """pcdl_commit / pcdl_open on the host cores at the small sizes (oracle: C MSM + the Python
    restatement of open_without_eval with the Poseidon transcript), and each size's GPU commitment
    checked against the oracle's (every size) -- added in place to `sweep`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pasta as P  # noqa: E402
    import pcdl_ref  # noqa: E402
    c = P.CURVES[cname]
    r = c.scalar
    S, Hp = (P.wrapped_to_point(c, [int(x) for x in q]) for q in (G[0], G[1]))
    toint = lambda a: P.from_mont(P.limbs_to_int(a), r)  # noqa: E731
    for lg, (p_, w_, z_, q_, wb_, C, pi) in inputs.items():
        e = sweep[f"2^{lg}"]
        pc = [toint(x) for x in p_]
        if lg <= 16:
            a0 = time.perf_counter()
            Cc = pcdl_ref.commit(cname, G, pc, toint(w_), S)
            e["cpu_commit_ms"] = (time.perf_counter() - a0) * 1e3
            e["commit_matches_cpu"] = bool(np.array_equal(np.array(P.point_to_wrapped(c, Cc), dtype=np.uint64), C))
        if lg <= 10:
            z = toint(z_)
            a0 = time.perf_counter()
            v = P.horner(pc, z, r)
            ref = pcdl_ref.open_without_eval(cname, pc, Cc, (1 << lg) - 1, z, v, G, S, Hp, w=toint(w_),
                                             q=[toint(x) for x in q_], w_bar=toint(wb_))
            e["cpu_open_ms"] = (time.perf_counter() - a0) * 1e3
            e["cpu_open_note"] = "Python restatement with C MSM/fold and the Poseidon sponge (not arkworks)"
            del ref
    return sweep


def _cpu_threads():
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    return min(threads, 16)


def cpu_ntt_baseline(L, H, logn, sp, gpu_ntt):
    """Rank 0, N=1 only: the C restatement of ark-poly's radix-2 FFT (oracle/oracle.c) on host cores,
    NTT + iNTT pair at the bench size, on the same input as one GPU forward transform (bit-exact check)."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import corc  # noqa: E402  (oracle: only the cpu_baseline legs may load it)

    N = 1 << logn
    rng = np.random.default_rng(7)
    x = rng.integers(0, 2**63, size=(N, 4), dtype=np.uint64)
    x[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    d = torch.from_numpy(x.view(np.int64).copy()).cuda()
    H.check(L.halo_ntt_dev(H.FP, ctypes.c_void_p(d.data_ptr()), logn, 1, 0, sp))
    torch.cuda.synchronize()
    y_gpu = d.cpu().numpy().view(np.uint64)
    threads = _cpu_threads()
    t0 = time.perf_counter()
    y = corc.ntt("fp", x, inverse=False, threads=threads)
    z = corc.ntt("fp", y, inverse=True, threads=threads)
    dt = time.perf_counter() - t0
    return {
        "workload": f"ntt+intt_2^{logn}_fp",
        "pair_ms": dt * 1e3,
        "elems_per_s_pair": N / dt,
        "cores": threads,
        "kind": "port",
        "sample": f"1 x NTT + iNTT at 2^{logn} (C restatement of ark-poly 0.5 radix-2 DIF/DIT + derange, OpenMP)",
        "gpu_matches_cpu": bool(np.array_equal(y, y_gpu)) and bool(np.array_equal(z, x)),
        "gpu_over_cpu": (dt * 1e3) / gpu_ntt["pair_ms"] if gpu_ntt else None,
    }


def cpu_prove_baseline(L, H, curve, cname, logn, gpu_out):
    """Rank 0, N=1 only: the same naive_prover pipeline on the C restatement backend
    (oracle/prover_ref.py CRefBackend over oracle.c, OpenMP) with the SRS the GPU run used; every
    commitment, evaluation and opening is compared with the GPU proof."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import prover_ref  # noqa: E402  (oracle: only the cpu_baseline legs may load it)

    from halo_amd import prover

    n = 1 << logn
    srs = np.zeros((n, 8), dtype=np.uint64)
    H.check(L.halo_srs_read(curve, 0, n, H.ptr(srs)))
    threads = _cpu_threads()
    B = prover_ref.CRefBackend(cname, srs, srs[1], threads=threads)
    wit = prover.synthetic_witness(B, n, seed=1)
    out = prover.naive_prover(B, wit, n, prover.Challenges(B.m))

    def same(a, b):
        return len(a) == len(b) and all(np.array_equal(x, y) for x, y in zip(a, b))

    ok = same(out["C_ws"], gpu_out["C_ws"]) and np.array_equal(out["C_z"], gpu_out["C_z"]) \
        and same(out["C_ts"], gpu_out["C_ts"]) and out["vs"] == gpu_out["vs"]
    for k in ("q_r", "q_r_omega", "acc"):
        a, b = out[k], gpu_out[k]
        ok = ok and np.array_equal(a["C"], b["C"]) and a["v"] == b["v"] and same(a["Ls"], b["Ls"]) \
            and same(a["Rs"], b["Rs"]) and np.array_equal(a["U"], b["U"]) and a["c"] == b["c"]
    return {
        "n": n,
        "ms": {k: v * 1e3 for k, v in out["times"].items()},
        "cores": threads,
        "kind": "port",
        "sample": f"1 x the naive_prover pipeline at 2^{logn} on the C restatement (ark-style NTT, Pippenger, "
                  f"per-element fold and division) with OpenMP",
        "gpu_matches_cpu": bool(ok),
    }


def cpu_fold_baseline(L, H, curve, logm, ipa):
    """Rank 0, N=1 only: one IPA fold round (pcdl.rs:427-435: G' = G_l + xi G_r with per-element
    scalar multiplication and affine conversion, c' and z' folds) over 2^logm element pairs, C
    restatement on host cores vs the device fold of the same inputs (halo_ipa_fold_host)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import corc  # noqa: E402  (oracle: only the cpu_baseline legs may load it)

    m = 1 << logm
    cname = "pallas" if curve == 0 else "vesta"
    gs = np.zeros((2 * m, 8), dtype=np.uint64)
    H.check(L.halo_srs_read(curve, 0, 2 * m, H.ptr(gs)))
    rng = np.random.default_rng(11)

    def fes(k):
        a = rng.integers(0, 2**63, size=(k, 4), dtype=np.uint64)
        a[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
        return np.ascontiguousarray(a)

    cs, zs, xi = fes(2 * m), fes(2 * m), fes(1)[0]
    xi_inv = corc.field_inv("fp" if curve == 0 else "fq", xi)
    g_gpu, c_gpu, z_gpu = gs.copy(), cs.copy(), zs.copy()
    H.check(L.halo_ipa_fold_host(curve, H.ptr(g_gpu), H.ptr(c_gpu), H.ptr(z_gpu), m, H.ptr(xi), H.ptr(xi_inv)))
    threads = _cpu_threads()
    t0 = time.perf_counter()
    g2, c2, z2 = corc.ipa_fold(cname, gs, cs, zs, xi, xi_inv, threads=threads)
    dt = time.perf_counter() - t0
    ok = np.array_equal(g2, g_gpu[:m]) and np.array_equal(c2, c_gpu[:m]) and np.array_equal(z2, z_gpu[:m])
    gpu_rate = None
    if ipa and ipa["glv_fold_path"]["fold_kernels_ms"]:
        # folds of G down to the tail threshold (lengths 2^logn .. 4096: 2^(logn-1) + ... + 2048 pairs)
        pairs = (1 << ipa["rounds"]) - 2048
        gpu_rate = pairs / (ipa["glv_fold_path"]["fold_kernels_ms"] * 1e-3)
    return {
        "workload": f"IPA fold round, {m} element pairs ({cname})",
        "elements_per_s": m / dt,
        "cores": threads,
        "kind": "port",
        "sample": f"1 x fold of 2^{logm} pairs (C restatement of pcdl.rs:427-435: per-element variable-base "
                  f"scalar multiplication + affine conversion), OpenMP",
        "gpu_matches_cpu": bool(ok),
        "gpu_elements_per_s": gpu_rate,
        "gpu_note": "device GLV fold kernels over the folded rounds of the 2^logn opening with "
                    "tuning ipa_weighted = 0 (extra.ipa_open.glv_fold_path); the default opening never folds G",
    }


if __name__ == "__main__":
    main()
