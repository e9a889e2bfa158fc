"""Kernel statistics from a rocprofv3 rocpd database (`--kernel-trace
--stats` without `--output-format csv` writes <name>_results.db): the
columns of rocprofv3's kernel_stats.csv plus the register / scratch figures
of each kernel.  Usage: rocpd_stats.py <results.db> <out.csv>"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                  "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(scratch_size), max(lds_size) "
                  "from kernels group by name order by sum(duration) desc").fetchall()
total = sum(r[2] for r in rows) or 1
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "VGPR", "AGPR",
                "SGPR", "ScratchBytes", "LdsBytes"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", f"{100.0 * r[2] / total:.3f}", r[4], r[5], r[6], r[7], r[8],
                    r[9], r[10]])
print(open(sys.argv[2]).read()[:1500])
