"""Print the render kernels of a rocprofv3 kernel trace as a timeline (ms from the first).
usage: python tools/trace_view.py TRACE.csv [first] [count]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(("k_", "void k_"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
a = int(sys.argv[2]) if len(sys.argv) > 2 else 0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 60
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[a:a + n]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    print(f"q{r['Queue_Id']:>2} s{r['Stream_Id']:>2} {name:16s} {s:9.3f} {e:9.3f} {e - s:6.3f}")
