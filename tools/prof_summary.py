"""Summarise a rocprofv3 kernel-trace database: per-kernel and per-(kernel, grid) time per step."""
import re
import sqlite3
import sys

db, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
con = sqlite3.connect(db)
cur = con.cursor()
rows = cur.execute("select name, count(*), sum(end-start), avg(end-start) from kernels group by name "
                   "order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total kernel time per step: {tot/1e6/steps:.2f} ms over {sum(r[1] for r in rows)/steps:.0f} launches")
for r in rows[:top]:
    nm = re.sub(r"\(.*", "", r[0]).replace("void sv::", "").replace("sv::", "")
    print(f"{r[2]/tot*100:6.2f}% {r[2]/steps/1e6:7.2f} ms/step n={r[1]/steps:6.1f} avg={r[3]/1e3:8.1f} us  {nm[:80]}")
if "--shapes" in sys.argv:
    rows = cur.execute("select name, grid_x, grid_y, grid_z, workgroup_x, count(*), sum(end-start), avg(end-start) "
                       "from kernels where name like '%gemm%' group by name, grid_x, grid_y, grid_z "
                       "order by sum(end-start) desc").fetchall()
    for r in rows[:top]:
        nm = re.sub(r"\(.*", "", r[0]).replace("void sv::", "")
        print(f"{r[6]/steps/1e3:8.1f} us/step n/step={r[5]/steps:4.1f} avg={r[7]/1e3:7.1f} us "
              f"wgs=({r[1]//r[4]},{r[2]},{r[3]}) {nm}")
