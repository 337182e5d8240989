"""Print one TD update's kernel timeline (start/end/duration in µs, queue) from a
rocprofv3 --kernel-trace CSV: the last complete update (agent_fwd to agent_fwd).
   python tools/timeline_trace.py <run_kernel_trace.csv>"""
import csv
import sys

r = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if "agent_fwd" in x["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
t0 = int(r[i0]["Start_Timestamp"])
print("queue   start_us    end_us    dur_us  kernel")
for x in r[i0:i1]:
    s, e = int(x["Start_Timestamp"]) - t0, int(x["End_Timestamp"]) - t0
    print(f"{x['Queue_Id']:>5} {s / 1000:9.1f} {e / 1000:9.1f} {(e - s) / 1000:9.1f}  {x['Kernel_Name'][:70]}")
print(f"update period: {(int(r[i1]['Start_Timestamp']) - t0) / 1000:.1f} us")
