# SQ counters (three passes) of the NTT pass kernels at 2^${1:-22} (tools/ntt_time.py: 11-bit passes up to 2^22, 8-bit above),
# run through gpurun from the repo root; per kernel: lane-instructions per element per pass, the VALU
# issue rate, the LDS-instruction share and the share of wave cycles waiting on LDS / anything.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_ntt; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $O/a -o run -- python3 tools/ntt_time.py ${1:-22} > $O/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM --output-format csv -d $O/b -o run -- python3 tools/ntt_time.py ${1:-22} > $O/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $O/c -o run -- python3 tools/ntt_time.py ${1:-22} > $O/c.log 2>&1 || exit 1
python3 - $O ${1:-22} <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ('a', 'b', 'c'):
    f = glob.glob(f'{O}/{sub}/**/*counter_collection.csv', recursive=True)[0]
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0]
        if 'ntt_pass' not in k: continue
        agg[k][r['Counter_Name'] + ('_c' if sub == 'c' and r['Counter_Name'] == 'SQ_WAVE_CYCLES' else '')].append(
            float(r['Counter_Value']))
for k, d in agg.items():
    c = {n: sum(v) / len(v) for n, v in d.items()}
    elems = 1 << int(sys.argv[2])  # per pass (one transform)
    cyc = c['GRBM_GUI_ACTIVE'] / 8
    print(k)
    print(f"  VALU lane-instructions per element per pass: {c['SQ_INSTS_VALU'] * 64 / elems:.0f}")
    print(f"  VALU wave-instructions per element: {c['SQ_INSTS_VALU'] / elems:.2f}; per wave: {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}")
    print(f"  VALU issue per CU per clock: {c['SQ_INSTS_VALU'] / (256 * cyc):.3f}; LDS instr per CU per clock: {c['SQ_INSTS_LDS'] / (256 * cyc):.3f}")
    print(f"  LDS bank conflict share: {100 * c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.1f} %")
    print(f"  wave cycles waiting on LDS: {100 * c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.1f} %, waiting on anything: {100 * c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.1f} %")
    wc = c.get('SQ_WAVE_CYCLES_c')
    if wc:
        print(f"  wave cycles (pass c): waiting {100 * c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES']:.1f} % (pass b), "
              f"issue-stalled {100 * c['SQ_WAIT_INST_ANY'] / wc:.1f} %, issuing {100 * c['SQ_ACTIVE_INST_ANY'] / wc:.1f} % "
              f"(VALU {100 * c['SQ_ACTIVE_INST_VALU'] / wc:.1f} %)")
    print(f"  raw: " + ", ".join(f"{n}={v:.0f}" for n, v in sorted(c.items())))
PY
rm -rf $O/a $O/b $O/c
