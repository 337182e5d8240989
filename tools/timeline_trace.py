"""Print one TD update's kernel timeline (start/end/duration in µs, queue) from a
rocprofv3 --kernel-trace CSV: the last complete update, from one launch of the
anchor kernel to the next (default agent_fwd; a pipelined update launches the agent
forward once per step range, so anchor it on the Adam kernel: `adam`).
   python tools/timeline_trace.py <run_kernel_trace.csv> [anchor]"""
import csv
import sys

r = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "agent_fwd"
idx = [i for i, x in enumerate(r) if anchor in x["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
t0 = int(r[i0]["Start_Timestamp"])
print("queue   start_us    end_us    dur_us  kernel")
for x in r[i0:i1]:
    s, e = int(x["Start_Timestamp"]) - t0, int(x["End_Timestamp"]) - t0
    print(f"{x['Queue_Id']:>5} {s / 1000:9.1f} {e / 1000:9.1f} {(e - s) / 1000:9.1f}  {x['Kernel_Name'][:70]}")
print(f"update period: {(int(r[i1]['Start_Timestamp']) - t0) / 1000:.1f} us")
