"""Timeline of a rocprofv3 rocpd database (kernels + memory copies), in start order:
relative start (ms), duration (ms), stream, name, grid / bytes.  Usage: trace_db.py DB [first] [count]"""
import sqlite3
import sys

db = sys.argv[1]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
c = sqlite3.connect(db)
ev = []
for n, s, e, g, st in c.execute("select s.kernel_name, k.start, k.end, k.grid_size_x, k.stream_id from rocpd_kernel_dispatch k "
                                "join rocpd_info_kernel_symbol s on k.kernel_id = s.id"):
    ev.append((s, e, st, n.split("(")[0][:40], "g=%d" % g))
for s, e, sz, st, nm in c.execute("select m.start, m.end, m.size, m.stream_id, m.name_id from rocpd_memory_copy m"):
    ev.append((s, e, st, "COPY", "%.2f MB" % (sz / 1e6)))
ev.sort()
t0 = ev[0][0]
for s, e, st, n, x in ev[first:first + count]:
    print("%9.3f %7.3f s%-3s %-40s %s" % ((s - t0) / 1e6, (e - s) / 1e6, st, n, x))
