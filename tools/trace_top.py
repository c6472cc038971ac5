"""Per-kernel call counts and mean durations (us) from a rocprofv3 rocpd database (--kernel-trace), filtered.
    python3 tools/trace_top.py <results.db> [substring ...]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    con = sqlite3.connect(sys.argv[1])
    keys = sys.argv[2:]
    agg = defaultdict(list)
    for name, dur in con.execute('select name, duration from kernels'):
        agg[name].append(dur)
    tot = sum(sum(v) for v in agg.values())
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if keys and not any(k in name for k in keys):
            continue
        print(f'{len(v):6d} {sum(v) / len(v) / 1e3:9.2f} us {sum(v) / tot * 100:5.2f} %  {name[:110]}')


if __name__ == '__main__':
    main()
