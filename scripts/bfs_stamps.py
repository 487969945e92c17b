"""Summarise the stage kernel's per-op stamps (-DBFS_STAMPS build, workgroup 0): per op the wall
cycles (wave 0's four segments), the slowest / fastest wave's compute segment and the stores."""
import collections, re, sys
d = collections.defaultdict(dict)
for l in open(sys.argv[1]):
    m = re.match(r'BFS op (\d+) w (\d+) comp (\d+) bar1 (\d+) store (\d+) bar2 (\d+)', l)
    if m:
        o, w, *v = map(int, m.groups())
        d[o][w] = v
tot = 0
for o in sorted(d):
    ws = d[o]
    wall = sum(ws[0])
    tot += wall
    print('op %2d wall %6d  comp max %6d min %6d  store max %6d' % (
        o, wall, max(v[0] for v in ws.values()), min(v[0] for v in ws.values()), max(v[2] for v in ws.values())))
print('total', tot)
