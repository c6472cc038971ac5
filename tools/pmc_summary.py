"""Per-kernel averages of every PMC counter in rocprofv3 rocpd databases.

    python tools/pmc_summary.py OUT.json DB [DB ...]
"""
import json
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, __import__('os').path.dirname(__file__))
from rocpd_report import short  # noqa: E402


def main():
    out, dbs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for db in dbs:
        c = sqlite3.connect(db)
        for name, cn, val in c.execute('select name, counter_name, counter_value from pmc_events'):
            acc[short(name)][cn].append(val)
    res = {k: {cn: sum(v) / len(v) for cn, v in sorted(d.items())} for k, d in acc.items()}
    with open(out, 'w') as f:
        json.dump(res, f, indent=1)
    for k, d in res.items():
        print(k)
        for cn, v in d.items():
            print(f'  {cn:32s} {v:16.1f}')


if __name__ == '__main__':
    main()
