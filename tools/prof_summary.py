"""Per-kernel summary of a rocprofv3 database (kernel-trace): calls, avg, share."""
import sqlite3
import sys


def main(path, top=20):
    cur = sqlite3.connect(path).cursor()
    rows = cur.execute("select name, count(*), avg(duration), sum(duration) from kernels group by name "
                       "order by sum(duration) desc").fetchall()
    tot = sum(r[3] for r in rows)
    print(f"{'calls':>7} {'avg_us':>9} {'share':>6}  kernel")
    for name, cnt, avg, sm in rows[:top]:
        print(f"{cnt:7d} {avg / 1000:9.2f} {100 * sm / tot:5.1f}%  {name.split('(')[0]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
