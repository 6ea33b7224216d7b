"""Markdown table from a rocprofv3 ``--stats`` kernel_stats.csv (per-step figures).

    python tools/stats_md.py <run_kernel_stats.csv> <steps profiled> "<title>" "<command>" [top]
"""
import csv
import re
import sys

path, steps, title, cmd = sys.argv[1], float(sys.argv[2]), sys.argv[3], sys.argv[4]
top = int(sys.argv[5]) if len(sys.argv) > 5 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# {title}\n")
print(f"Command: `{cmd}`")
print(f"Total kernel time {tot / 1e6:.1f} ms over {steps:.0f} steps = {tot / 1e6 / steps:.2f} ms/step.\n")
print("| % | ms/step | calls/step | avg us | kernel |")
print("|---|---|---|---|---|")
for r in rows[:top]:
    nm = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")
    print(f"| {float(r['Percentage']):.1f} | {float(r['TotalDurationNs']) / 1e6 / steps:.2f} | "
          f"{int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | `{nm}` |")
