#!/usr/bin/env python3
"""Milestones of one encode step from rocprofv3 kernel traces (tools/kt_ab.sh), side by side:
per-stream busy time and the start / end of the kernels that bound the sort stream's phases
(Lyndon spans / merge, round 0, doubling rounds, BBWT gather, MTF) and of the LZ77 parse.

    python tools/kt_steps.py OUT/TAG/kt_kernel_trace.csv [...]

A step ends at its k_mdl launch; the second step of the trace (the timed one) is shown.
"""
import csv, sys, collections
def load(path):
    rows=[]
    with open(path) as f:
        for r in csv.DictReader(f):
            n=r["Kernel_Name"].replace("(anonymous namespace)::","").replace("kolm::","")
            if n.startswith("void "): n=n[5:]
            n=n.split("(")[0]
            rows.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),n,r.get("Stream_Id") or r.get("Queue_Id")))
    rows.sort()
    return rows
def steps(rows):
    ends=[i for i,r in enumerate(rows) if r[2].startswith("k_mdl")]
    st=[0]+[e+1 for e in ends[:-1]]
    return [(s,e) for s,e in zip(st,ends)]
for path in sys.argv[1:]:
    rows=load(path); ss=steps(rows)
    s,e=ss[1]  # the timed step
    # extend to include emission after mdl
    seg=rows[s:e+8]
    t0=seg[0][0]
    byq=collections.defaultdict(list)
    for r in seg: byq[r[3]].append(r)
    print(path, "steps", len(ss), "step span ms", (rows[e][1]-t0)/1e6)
    for q,rs in byq.items():
        busy=sum(r[1]-r[0] for r in rs)/1e6
        print("  stream",q,"kernels",len(rs),"busy",round(busy,2),"first",round((rs[0][0]-t0)/1e6,2),"last end",round((rs[-1][1]-t0)/1e6,2), collections.Counter(r[2] for r in rs).most_common(3))
    # milestones
    def last_end(prefix): 
        v=[r[1] for r in seg if r[2].startswith(prefix)]; return round((max(v)-t0)/1e6,2) if v else None
    def first_start(prefix):
        v=[r[0] for r in seg if r[2].startswith(prefix)]; return round((min(v)-t0)/1e6,2) if v else None
    for k in ["k_duval_span","k_duval_merge","k_fsfl","k_alpha_codes","k_keypos_r0","k_r0_rk","k_classify","k_bbwt_gather","k_mtf_summary","k_mtf_replay","k_lz_tiles","k_lz_local","k_lz_stitch","k_mdl"]:
        print(f"   {k:18s} start {first_start(k)} end {last_end(k)}")
