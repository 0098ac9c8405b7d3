#!/usr/bin/env python3
"""Host/device timeline of one bench step from a rocprofv3 CSV trace
(--hip-trace --kernel-trace --memory-copy-trace, tools/gpu_run.sh apitrace):
the HIP calls of the main thread and the kernels / copies, in time order,
for the STEP-th glp_simplex call inside the k_gk_mark window, with the GPU's
idle gaps and the host's time between calls.
usage: api_timeline.py DIR [STEP]"""
import csv
import os
import sys

d = sys.argv[1]
step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
api = list(csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))))
ker = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
cpy = list(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))))
marks = sorted(int(k["Start_Timestamp"]) for k in ker if k["Kernel_Name"].startswith("k_gk_mark"))
t0, t1 = marks[0], marks[1]
main_tid = max(set(a["Thread_Id"] for a in api), key=lambda t: sum(1 for a in api if a["Thread_Id"] == t))
ev = []
for a in api:
    s_, e_ = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    if t0 <= s_ <= t1 and a["Thread_Id"] == main_tid:
        ev.append((s_, e_, "H", a["Function"]))
for k in ker:
    s_, e_ = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    if t0 <= s_ <= t1:
        ev.append((s_, e_, "K", k["Kernel_Name"].split("(")[0][:60]))
for c in cpy:
    s_, e_ = int(c["Start_Timestamp"]), int(c["End_Timestamp"])
    if t0 <= s_ <= t1:
        ev.append((s_, e_, "C", c["Direction"].replace("MEMORY_COPY_", "")))
ev.sort()
# steps: split at the big host gaps (the bench's Python between calls) -> use
# the k_dual_finish kernels as call ends? simplest: split by hipGraphLaunch groups
gpu = sorted((s_, e_) for s_, e_, k, _ in ev if k in "KC")
busy, last = 0, None
for s_, e_ in gpu:
    if last is None or s_ > last:
        busy += e_ - s_ if last is None or s_ >= last else e_ - last
        last = e_
    elif e_ > last:
        busy += e_ - last
        last = e_
span = t1 - t0
print(f"window {span / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us ({100 * busy / span:.1f}%)")
# host call totals by function
tot = {}
for s_, e_, k, nm in ev:
    if k == "H":
        c = tot.setdefault(nm, [0, 0])
        c[0] += 1
        c[1] += e_ - s_
for nm, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:20]:
    print(f"  {nm:40s} {n:6d} calls {t / 1e3:9.1f} us")
# idle GPU gaps > 5 us with the host calls inside them
print("GPU idle gaps > 5 us (and the host calls during them):")
last = t0
gi = 0
for s_, e_ in gpu:
    if s_ - last > 5000:
        inside = [nm for (hs, he, k, nm) in ev if k == "H" and hs < s_ and he > last]
        gi += s_ - last
        print(f"  {(last - t0) / 1e3:9.1f} +{(s_ - last) / 1e3:7.1f} us: {', '.join(inside[:8])}{' ...' if len(inside) > 8 else ''}")
    last = max(last, e_)
print(f"idle in gaps > 5 us: {gi / 1e3:.1f} us")

if len(sys.argv) > 4:
    a_, b_ = float(sys.argv[3]) * 1e3 + t0, float(sys.argv[4]) * 1e3 + t0
    for s_, e_, k, nm in ev:
        if a_ <= s_ <= b_ and nm not in ("__hipPushCallConfiguration", "__hipPopCallConfiguration"):
            print(f"{(s_ - t0) / 1e3:9.1f} {(e_ - s_) / 1e3:7.1f} {k} {nm}")
