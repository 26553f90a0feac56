#!/usr/bin/env python3
"""Per-stream timeline of one encode step from a rocprofv3 kernel trace.

    python tools/timeline.py OUT/kt/kt_kernel_trace.csv [--step -1]

A step starts at a k_iota dispatch on the main stream that follows the previous
step's last emission kernel; each step is split into phases at the sort-pass
boundaries (k_iota) and the per-stream busy time, idle gaps and the top kernels of
every phase are printed, so the critical path of the two-stream pipeline is visible.
"""
import argparse
import csv
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("kolm::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-1)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Stream_Id", r.get("Queue_Id"))))
    rows.sort()
    # a step = from a k_lz_emit-free region start; split on the MDL kernel (one per step)
    ends = [i for i, r in enumerate(rows) if r[2].startswith("k_mdl")]
    starts = [0] + [e + 1 for e in ends[:-1]]
    steps = []
    for s, e in zip(starts, ends):
        # extend to the emission kernels after the MDL
        j = e + 1
        while j < len(rows) and (rows[j][2].startswith("k_emit") or rows[j][2].startswith("k_rice_emit")
                                 or rows[j][2].startswith("k_lz_emit") or rows[j][2].startswith("k_simple")
                                 or rows[j][2].startswith("k_offsets")):
            j += 1
        steps.append(rows[s:j])
    print(f"{len(steps)} steps in trace")
    st = steps[a.step]
    t0 = st[0][0]
    t1 = max(r[1] for r in st)
    print(f"step span {(t1 - t0) / 1e6:.2f} ms, {len(st)} kernels")
    by_stream = defaultdict(list)
    for r in st:
        by_stream[r[3]].append(r)
    for sid, rs in sorted(by_stream.items()):
        busy = sum(r[1] - r[0] for r in rs)
        print(f"stream {sid}: {len(rs)} kernels, busy {busy / 1e6:.2f} ms, first {(rs[0][0] - t0) / 1e6:.2f}"
              f" last-end {(max(r[1] for r in rs) - t0) / 1e6:.2f} ms")
    # phases on each stream, split where one of the marker kernels starts
    print("\nper-stream phases:")
    marks = ("k_iota", "k_duval_span", "k_lz_local", "k_prevc", "k_mtf_summary", "k_sizes")
    for sid, rs in sorted(by_stream.items()):
        phases = []
        for r in rs:
            if not phases or any(r[2].startswith(m) for m in marks):
                phases.append([r[2], r[0], r[1], defaultdict(float), 0])
            cur = phases[-1]
            cur[2] = max(cur[2], r[1])
            cur[3][r[2]] += (r[1] - r[0]) / 1e6
            cur[4] += 1
        for name, s0, e0, ks, n in phases:
            top = sorted(ks.items(), key=lambda kv: -kv[1])[:6]
            print(f"  [{sid}] {name:16s} {(s0 - t0) / 1e6:7.2f} -> {(e0 - t0) / 1e6:7.2f} ms "
                  f"({(e0 - s0) / 1e6:6.2f} wall, {sum(ks.values()):6.2f} busy, {n:3d} k): "
                  + ", ".join(f"{k} {v:.2f}" for k, v in top))
    # gaps on the last-finishing stream
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in st:
        tot[r[2]] += (r[1] - r[0]) / 1e6
        cnt[r[2]] += 1
    print("\nkernel totals (ms, launches):")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:30]:
        print(f"  {k:34s} {v:8.3f} {cnt[k]:5d}  avg {v / cnt[k] * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
