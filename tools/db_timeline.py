#!/usr/bin/env python3
"""Per-stream timeline of the last k_repair-containing step from a rocprofv3 sqlite db.

    python tools/db_timeline.py OUT/tr/x_results.db
"""
import sqlite3
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("kolm::", "")
    return (n[5:] if n.startswith("void ") else n).split("(")[0]


c = sqlite3.connect(sys.argv[1])
rows = c.execute("select d.start, d.end, d.stream_id, d.queue_id, k.kernel_name from rocpd_kernel_dispatch d "
                 "join rocpd_info_kernel_symbol k on d.kernel_id = k.id order by d.start").fetchall()
rep = [r for r in rows if "k_repair" in r[4]]
r0 = rep[-1]
t0 = r0[0]
# the step: from the memset/first kernel before the last k_repair to the last emission kernel
win = [r for r in rows if r[0] >= t0 - 2e6 and r[0] <= r0[1] + 200e6]
print(f"k_repair {(r0[1] - r0[0]) / 1e6:.2f} ms")
by = {}
for s, e, st, q, n in win:
    by.setdefault(q, []).append((s, e, short(n)))
for q, L in by.items():
    busy = sum(e - s for s, e, _ in L) / 1e6
    print(f"queue {q}: {len(L)} kernels, first start {(L[0][0] - t0) / 1e6:.2f} ms, last end {(L[-1][1] - t0) / 1e6:.2f} ms, busy {busy:.2f} ms")
    agg = {}
    for s, e, n in L:
        a = agg.setdefault(n, [0, 0.0, 1e30, 0])
        a[0] += 1
        a[1] += (e - s) / 1e6
        a[2] = min(a[2], (s - t0) / 1e6)
        a[3] = max(a[3], (e - t0) / 1e6)
    for n, (k, ms, st, en) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
        print(f"    {n[:60]:60s} x{k:3d} {ms:8.2f} ms  [{st:8.2f} .. {en:8.2f}]")
