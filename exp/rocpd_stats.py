"""Kernel statistics (calls, total/avg ms) from a rocprofv3 rocpd SQLite
database, for runs made without --output-format csv."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("""
    select s.display_name, count(*), sum(d.end - d.start), avg(d.end - d.start)
    from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
    group by s.display_name order by sum(d.end - d.start) desc""").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'kernel':70s} {'calls':>6s} {'total ms':>9s} {'avg ms':>8s} {'%':>5s}")
for name, n, t, a in rows:
    print(f"{name[:70]:70s} {n:6d} {t / 1e6:9.3f} {a / 1e6:8.4f} {100 * t / tot:5.1f}")
