#!/usr/bin/env python3
"""GPU busy fraction and idle gaps of a run from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d out -o e -- python3 bench_enrich.py ...
    python scripts/kernel_gaps.py out/.../e_kernel_trace.csv [elapsed_s]

``elapsed_s``: only the last that many seconds of the trace (the timed run
at the end of a bench process); busy = the union of kernel intervals.  The
largest gaps are listed by the kernels around them.
"""
import csv, sys, collections, json, re
rows = list(csv.DictReader(open(sys.argv[1])))
elapsed_ms = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else None
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t_end = max(e for _, e, _ in ev)
t_beg = t_end - elapsed_ms * 1e6 if elapsed_ms else ev[0][0]
ev = [x for x in ev if x[0] >= t_beg]
busy = 0
cur_s, cur_e = ev[0][0], ev[0][1]
gaps = []
prev_name = ev[0][2]
for s, e, n in ev[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, n, prev_name, cur_e - ev[0][0]))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n
busy += cur_e - cur_s
wall = t_end - ev[0][0]
print(f"window (timed run, last {wall/1e6:.1f} ms)  busy {busy/1e6:.1f} ms ({100*busy/wall:.1f}%)  kernels {len(ev)}")
hist, tot = collections.Counter(), collections.Counter()
for g, n, p, _ in gaps:
    b = "<2us" if g < 2e3 else "2-5us" if g < 5e3 else "5-20us" if g < 20e3 else "20-100us" if g < 1e5 else "100us-1ms" if g < 1e6 else ">1ms"
    hist[b] += 1
    tot[b] += g
for b in ["<2us", "2-5us", "5-20us", "20-100us", "100us-1ms", ">1ms"]:
    print(f"  gaps {b:>9}: {hist[b]:6d}  total {tot[b]/1e6:8.1f} ms")
big = collections.Counter()
for g, n, p, _ in gaps:
    if g >= 2e4:
        big[(p[:50], n[:50])] += g
for (p, n), g in big.most_common(10):
    print(f"  >20us gaps {g/1e6:7.1f} ms  after [{p}]  before [{n}]")
for g, n, p, t in sorted(gaps, reverse=True)[:8]:  # the largest single gaps, where in the window
    if g >= 5e5:
        print(f"  gap {g/1e6:7.2f} ms at {t/1e6:8.1f} ms  after [{p[:50]}]  before [{n[:50]}]")
