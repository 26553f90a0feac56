#!/usr/bin/env python3
"""Kernel-by-kernel listing of one batch from a rocprofv3 kernel trace (tools/gpu_call.sh probe:KIND):
start offset, duration and the idle gap before each kernel, per queue, for the last batch in the trace
(batches split at k_mdl).  BATCH counts from the end (default 2: lz_probe.py times the kernels of its
last batch with events, which add gaps; the one before is untimed).

    python tools/kt_list.py OUT/probe_KIND/kt_kernel_trace.csv [BATCH] [queue]
"""
import csv
import sys


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("kolm::", "")
            n = (n[5:] if n.startswith("void ") else n).split("(")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r.get("Queue_Id") or r.get("Stream_Id")))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if r[2].startswith("k_mdl")]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    s = ends[-back - 1] + 1 if len(ends) > back else 0
    seg = rows[s:ends[-back + 1] + 1] if back > 1 else rows[s:]
    t0 = seg[0][0]
    queues = sorted({r[3] for r in seg})
    want = sys.argv[3] if len(sys.argv) > 3 else None
    for q in queues:
        if want and q != want:
            continue
        rs = [r for r in seg if r[3] == q]
        print(f"queue {q}: {len(rs)} kernels, busy {sum(r[1] - r[0] for r in rs) / 1e6:.3f} ms")
        prev = None
        for r in rs:
            gap = (r[0] - prev) / 1e3 if prev is not None else 0.0
            print(f"  {(r[0] - t0) / 1e6:8.3f} ms  {(r[1] - r[0]) / 1e3:8.1f} us  gap {gap:6.1f} us  {r[2]}")
            prev = r[1]


if __name__ == "__main__":
    main()
