"""Summarise kernel dispatches of a rocprofv3 rocpd sqlite database (per-kernel count/total/avg)."""
import glob
import sqlite3
import sys

db = sys.argv[1]
if not db.endswith(".db"):
    db = glob.glob(db + "/**/*.db", recursive=True)[0]
con = sqlite3.connect(db)
cur = con.cursor()
tabs = {r[0].split("_0")[0]: r[0] for r in cur.execute("select name from sqlite_master where type='table'")}
kd, ks = tabs["rocpd_kernel_dispatch"], tabs["rocpd_info_kernel_symbol"]
cols = [r[1] for r in cur.execute(f"pragma table_info({kd})")]
scols = [r[1] for r in cur.execute(f"pragma table_info({ks})")]
name_col = "kernel_name" if "kernel_name" in scols else ("display_name" if "display_name" in scols else scols[1])
rows = cur.execute(f"select s.{name_col}, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.start), max(d.end) "
                   f"from {kd} d join {ks} s on d.kernel_id = s.id group by s.{name_col} order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
span = (max(r[5] for r in rows) - min(r[4] for r in rows)) if rows else 0
print(f"{'kernel':60s} {'calls':>8s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for r in rows:
    print(f"{r[0][:60]:60s} {r[1]:8d} {r[2] / 1e6:10.3f} {r[3] / 1e3:9.2f} {100 * r[2] / tot:6.1f}")
print(f"TOTAL kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches; wall span {span / 1e6:.1f} ms")
