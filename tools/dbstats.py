"""Per-kernel stats from a rocprofv3 rocpd sqlite database (when csv output was not requested)."""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("""select s.display_name, count(*), sum(d.end - d.start), avg(d.end - d.start)
                    from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
                    group by s.display_name order by 3 desc""").fetchall()
tot = sum(r[2] for r in rows)
print(f"total {tot/1e6:.1f} ms")
for n, k, t, a in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{n[:70]:70s} {k:>5} {t/1e6:9.2f} ms {a/1e3:9.1f} us")
