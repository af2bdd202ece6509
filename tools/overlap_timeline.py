"""Timeline of learner ticks from a rocprofv3 kernel-trace csv: the kernels
around the middle acting launch (the kernel whose name holds `key`, default
act_step), start / end relative to it (us) and queue, plus over all acting
launches in the middle half: the median tick period and the median time
another kernel ran beside the acting launch.

    python tools/overlap_timeline.py kernel_trace.csv [n_kernels] [key]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
key = sys.argv[3] if len(sys.argv) > 3 else "act_step"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
S = [int(r["Start_Timestamp"]) for r in rows]
E = [int(r["End_Timestamp"]) for r in rows]
acts = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
if not acts:
    acts = [i for i, r in enumerate(rows) if "k_step" in r["Kernel_Name"]]
mid = acts[len(acts) // 2]
t0 = S[mid]
q = next((c for c in ("Queue_Id", "Stream_Id") if c in rows[0]), None)
for i in range(max(0, mid - 3), min(len(rows), mid + n)):
    r = rows[i]
    print(f'{(S[i] - t0) / 1e3:9.2f} {(E[i] - t0) / 1e3:9.2f} {(E[i] - S[i]) / 1e3:7.2f}  '
          f'q={r.get(q, "?") if q else "?":>3}  {r["Kernel_Name"][:80]}')
sel = acts[len(acts) // 4: 3 * len(acts) // 4]
period = statistics.median([(S[b] - S[a]) / 1e3 for a, b in zip(sel, sel[1:])])
beside = []
for a in sel:
    ov = 0
    for j in range(max(0, a - 40), min(len(rows), a + 40)):
        if j != a:
            ov = max(ov, min(E[a], E[j]) - max(S[a], S[j]))
    beside.append(ov / 1e3)
print(f"acting launches {len(acts)}; median tick period {period:.2f} us; acting launch "
      f"{statistics.median([(E[a] - S[a]) / 1e3 for a in sel]):.2f} us, longest overlap with another kernel "
      f"(median) {statistics.median(beside):.2f} us")
