"""Print per-dispatch kernel durations from a rocprofv3 rocpd database (last N dispatches)."""
import glob
import sqlite3
import sys

f = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
c = sqlite3.connect(f)
rows = c.execute('select name, duration, grid_x, workgroup_x, lds_size, vgpr_count from kernels order by start').fetchall()
tot = 0
for name, d, g, wg, lds, v in rows[-n:]:
    tot += d
    print('%9.1f us  grid %7d wg %4d lds %6d vgpr %3d  %s' % (d / 1e3, g // max(wg, 1), wg, lds, v, name[:90]))
print('total %.1f us' % (tot / 1e3))
