"""Summarise rocprofv3 rocpd databases into committed profile artefacts.

  python tools/rocpd_report.py --trace gpurun_out/prof_r01/trace_results.db \
      --fetch gpurun_out/pmc_fetch_r01/fetch_results.db --write gpurun_out/pmc_write_r01/write_results.db \
      --tag r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats
equivalent: calls, total/avg/min/max ns per kernel) and profiles/<tag>_pmc.json
(per-kernel average HBM bytes per launch). FETCH_SIZE is reported in KiB and,
on gfx950, counts half the bytes of wide (16 B/lane) coalesced reads
(MI355X_MICROARCH.md §HBM), so read bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE
(KiB) is exact for 16-B streaming stores and uncalibrated for narrower ones
(our conv epilogue stores 4 B per lane), which the JSON records.
"""
import argparse
import csv
import json
import os
import sqlite3
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    # 'void dm::(anonymous namespace)::conv_igemm_kernel<128, 128, 64, 64, 0>(dm::ConvArgs)' -> conv_igemm_kernel<128,128,64,64,0>
    n = name.replace('void ', '').replace('dm::(anonymous namespace)::', '')
    if '(' in n:
        n = n[:n.index('(')]
    return n.replace(' ', '')


def kernel_stats(db):
    c = sqlite3.connect(db)
    agg = defaultdict(list)
    for name, dur in c.execute('select name, duration from kernels'):
        agg[name].append(dur)
    rows = []
    total = sum(sum(v) for v in agg.values())
    for name, d in agg.items():
        rows.append(dict(Name=name, Calls=len(d), TotalDurationNs=sum(d), AverageNs=sum(d) / len(d),
                         Percentage=100.0 * sum(d) / total, MinNs=min(d), MaxNs=max(d)))
    rows.sort(key=lambda r: -r['TotalDurationNs'])
    return rows


def calls_by_name(db):
    c = sqlite3.connect(db)
    agg = defaultdict(int)
    for (name, ) in c.execute('select name from kernels'):
        agg[short(name)] += 1
    return agg


def pmc(db, counter):
    c = sqlite3.connect(db)
    agg = defaultdict(list)
    for name, val in c.execute('select name, counter_value from pmc_events where counter_name = ?', (counter, )):
        agg[name].append(val)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trace', required=True)
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    ap.add_argument('--tag', default='r01')
    ap.add_argument('--command', default='')
    ap.add_argument('--workload', default='c3')
    ap.add_argument('--build', default=None, help='dm_build_info() of the library the passes ran')
    args = ap.parse_args()
    out_dir = os.path.join(ROOT, 'profiles')
    os.makedirs(out_dir, exist_ok=True)
    rows = kernel_stats(args.trace)
    path = os.path.join(out_dir, f'{args.tag}_kernel_stats.csv')
    # (the workload is in the tag of the run's files; the CSV keeps rocprofv3's --stats columns)
    with open(path, 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    print('wrote', path)
    for r in rows[:12]:
        print(f"{short(r['Name']):50s} calls {r['Calls']:6d} avg {r['AverageNs'] / 1e3:9.1f} us  {r['Percentage']:5.1f}%")
    if args.fetch and args.write:
        fetch = pmc(args.fetch, 'FETCH_SIZE')
        write = pmc(args.write, 'WRITE_SIZE')
        res = {}
        # launches per forward of each kernel in the FETCH pass: its dispatches over the timestep embedding's (one per
        # network forward, the plan-building forward included); bench.py's roofline takes this summary's traffic only
        # for the same build and the same count
        calls = calls_by_name(args.fetch)
        fwds = calls.get('timestep_embed_kernel', 0)
        for name in set(fetch) | set(write):
            rb = 2 * 1024 * fetch.get(name, 0.0)
            wb = 1024 * write.get(name, 0.0)
            k = short(name)
            res[k] = dict(read_bytes_per_launch=rb, write_bytes_per_launch=wb, hbm_bytes_per_launch=rb + wb,
                          fetch_size_kib=fetch.get(name), write_size_kib=write.get(name), calls=calls.get(k, 0),
                          launches_per_forward=(calls.get(k, 0) / fwds) if fwds else None)
        meta = dict(note='read = 2 x FETCH_SIZE (gfx950 half-count of 16B/lane coalesced reads); '
                         'write = WRITE_SIZE (exact for 16B stores, uncalibrated for 4B stores)',
                    command=args.command, workload=args.workload, build=args.build, forwards=fwds, kernels=res)
        path = os.path.join(out_dir, f'{args.tag}_pmc.json')
        with open(path, 'w') as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print('wrote', path)
        for k, v in sorted(res.items(), key=lambda kv: -kv[1]['hbm_bytes_per_launch'])[:8]:
            print(f'{k:50s} read {v["read_bytes_per_launch"] / 1e6:9.2f} MB  write {v["write_bytes_per_launch"] / 1e6:9.2f} MB')


if __name__ == '__main__':
    main()
