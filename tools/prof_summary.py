"""Summarise a rocprofv3 kernel trace: per-kernel totals per step and the per-step span/gap breakdown."""
import collections
import csv
import glob
import os
import sqlite3
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 24
traces = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
if traces:
    rows = [r for t in traces for r in csv.DictReader(open(t))]
else:  # rocprofv3's default rocpd (SQLite) output
    db = sqlite3.connect(glob.glob(f"{d}/**/*.db", recursive=True)[0])
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
            for n, s, e in db.execute("select name, start, end from kernels")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tot = collections.defaultdict(float)
cnt = collections.Counter()
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]
    tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[n] += 1
# steady state: the last 10 complete steps (windows between consecutive gather launches)
gi = [i for i, r in enumerate(rows) if "gather_batch" in r["Kernel_Name"]]
if len(gi) >= 12:
    win = rows[gi[-11]:gi[-1]]
    wt = collections.defaultdict(float)
    wc = collections.Counter()
    for r in win:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]
        wt[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        wc[n] += 1
    WS = sum(wt.values())
    span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
    print(f"steady state (last 10 steps): {len(win) / 10:.0f} kernels/step, busy {WS / 10:.1f} us/step, "
          f"span {span / 10:.1f} us/step")
    for n, t in sorted(wt.items(), key=lambda x: -x[1])[:30]:
        print(f"{t / 10:8.1f} us/step {100 * t / WS:5.1f}%  {wc[n] / 10:5.1f} calls/step  {t / wc[n]:6.1f} us/call  {n}")
    print()
S = sum(tot.values())
print(f"kernel time total {S/1e3:.2f} ms over {steps} steps -> {S/steps:.1f} us/step")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:25]:
    print(f"{t/steps:8.1f} us/step {100*t/S:5.1f}%  {cnt[n]/steps:5.1f} calls/step  {t/cnt[n]:6.1f} us/call  {n}")
# last step window: kernels after the last gather_batch
idx = [i for i, r in enumerate(rows) if "gather_batch" in r["Kernel_Name"]]
if len(idx) >= 2:
    w = rows[idx[-2]:idx[-1]]
    span = (int(w[-1]["End_Timestamp"]) - int(w[0]["Start_Timestamp"])) / 1e3
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in w) / 1e3
    print(f"one step: {len(w)} kernels, span {span:.1f} us, busy {busy:.1f} us, gaps {span-busy:.1f} us")
