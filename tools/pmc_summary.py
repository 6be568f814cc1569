"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per dispatch, per kernel.

usage: python tools/pmc_summary.py <dir-with-counter_collection.csv> [...]
"""
import collections, csv, glob, os, sys

def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows

def summarise(rows):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for r in rows:
        k = r.get('Kernel_Name') or r.get('Kernel-Name') or r.get('kernel_name')
        c = r.get('Counter_Name') or r.get('Counter-Name')
        v = float(r.get('Counter_Value') or r.get('Counter-Value') or 0)
        dsp = r.get('Dispatch_Id') or r.get('Dispatch-Id') or r.get('Correlation_Id')
        acc[k][c] += v
        disp[k][c].add(dsp)
    out = {}
    for k in acc:
        out[k] = {c: acc[k][c] / max(1, len(disp[k][c])) for c in acc[k]}
        out[k]['dispatches'] = max(len(s) for s in disp[k].values())
    return out

if __name__ == '__main__':
    res = {}
    for d in sys.argv[1:]:
        for k, v in summarise(load(d)).items():
            res.setdefault(k, {}).update(v)
    for k in sorted(res, key=lambda k: -max(v for c, v in res[k].items() if c != 'dispatches')):
        short = k.split('(')[0][-48:]
        print('%-48s %s' % (short, '  '.join('%s=%.4g' % (c, v) for c, v in sorted(res[k].items()))))
