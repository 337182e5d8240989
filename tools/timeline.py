"""One update's kernel timeline from a rocprofv3 kernel trace (the last complete
update of the run): start / end / duration (us) and queue per kernel.
    python tools/timeline.py <run_kernel_trace.csv>"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "agent_fwd" in r["Kernel_Name"]]
    i0, i1 = idx[-2], idx[-1]
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:70]}")
    print("update:", (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3, "us")


if __name__ == "__main__":
    main(sys.argv[1])
